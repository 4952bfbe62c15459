// Grouped positional convolution of wav2vec2 (Wav2Vec2PositionalConvEmbedding: Conv1d(D, D, 128,
// padding 64, groups 16) + SamePad + GELU, residual add; modeling_wav2vec2.py, called from
// src/model/w2v_custom_feat_extractor.py via the encoder) on bf16 MFMA, three kernels:
//
//   pc16_k<false>  forward:  xsum = gelu(conv(e) + bias) + e, pre = conv(e) + bias, e16 = bf16(e)
//   pc16_k<true>   backward-data: dpre = dxsum * gelu'(pre) (formed while staged), de = convT(dpre) + dxsum,
//                  dpre16 = bf16(dpre), per-sample column sums of dpre (conv-bias gradient)
//   pc16_wgrad_k   weight gradient: dW[o][tap][i] = sum_{b,t} dpre[b,t,o] * e[b, t+tap-64, i]
//
// A GEMM view of this conv (M = B*T tokens, N = 48 channels of a group, K = 128 taps x 48) re-reads
// every input frame 128 times through the implicit-conv operand and leaves 3/8 of a 128-wide tile
// idle. Here one workgroup owns a (group, pair of samples): the two samples' input frames
// [-pad, T+127-pad) x 48 channels are staged in LDS ONCE (bf16, 112-B rows: conflict-free 16-row
// fragment reads), the group's weights stream through LDS in 4-tap chunks (LDS-DMA, double
// buffered), and every MFMA A fragment is a shifted row window of the staged slab. 8 waves: wave w
// computes sample w/4, output rows 64*(w%4) .. +63, all 48 output channels (4 x 3 MFMA tiles).
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {

constexpr int PC_G = 48;                       // channels per group (wav2vec2-base: 768 / 16)
constexpr int PC_TAPS = 128;
constexpr int PC_KT = PC_TAPS * PC_G;          // 6144: reduction length per output channel
constexpr int PC_TC = 4;                       // taps per weight chunk
constexpr int PC_NCH = PC_TAPS / PC_TC;        // 32 chunks
constexpr int PC_XLD = 56;                     // slab row stride (bf16) = 112 B
constexpr int PC_WPR = PC_TC * PC_G / 8 + 1;   // 16-B pieces per weight-chunk row: 24 + 1 pad = 25 (400 B)
constexpr int PC_WIN = 24;                     // glds wave-instructions per weight chunk (1536 pieces >= 48 x 25)
constexpr int PC_WBUF = PC_WIN * 1024;         // 24 KB per weight buffer
constexpr int PC_TMAX = 256;
constexpr int PC_SLAB = (PC_TMAX + PC_TAPS - 1) * PC_XLD * 2;   // 42896 B per sample
constexpr int PC_LDS = 2 * PC_WBUF + 2 * PC_SLAB;              // 134944 B

__device__ __attribute__((aligned(16))) uint32_t g_pc_zero[8];

typedef __attribute__((address_space(3))) void lds_t;
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const void* src, lds_t* dst) {
  __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
}

// workgroup -> (group, sample pair), XCD-aware: the blocks that share an XCD (blockIdx % 8) get a
// contiguous range, so the workgroups of one group (same weights) share an L2
__device__ __forceinline__ int xcd_linear(int orig, int nwg) {
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
}

// this wave's 3 LDS-DMA pieces of weight chunk `ch` (rows r = 0..47 of the group's image, 25
// pieces a row, the last a zero pad) into `buf`
__device__ __forceinline__ void issue_wchunk(const uint16_t* __restrict__ wimg, int g, int ch, char* buf, int wave,
                                             int lane) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int j = wave * 3 + i;
    const int q = j * 64 + lane;
    const int row = q / PC_WPR, p = q - row * PC_WPR;
    const void* src = (row < PC_G && p < PC_WPR - 1)
                          ? (const void*)(wimg + ((int64_t)(g * PC_G + row) * PC_KT + ch * (PC_TC * PC_G) + 8 * p))
                          : (const void*)g_pc_zero;
    glds16(src, (lds_t*)(buf + j * 1024));
  }
}

template <bool BWD>
__global__ void __launch_bounds__(512, 1) pc16_k(const float* __restrict__ x, const float* __restrict__ pre_in,
                                                 const uint16_t* __restrict__ wimg, const float* __restrict__ bias,
                                                 float* __restrict__ out, float* __restrict__ pre_out,
                                                 uint16_t* __restrict__ side16, float* __restrict__ colpart, int B,
                                                 int T, int D, int pad, int npairs) {
  __shared__ __attribute__((aligned(1024))) char smem[PC_LDS];
  uint16_t* slab = reinterpret_cast<uint16_t*>(smem + 2 * PC_WBUF);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lin = xcd_linear(blockIdx.x, gridDim.x);
  const int g = lin / npairs, pair = lin - g * npairs;
  const int nrows = T + PC_TAPS - 1;

  issue_wchunk(wimg, g, 0, smem, wave, lane);

  // ---- stage both samples' frames (bf16) + side outputs (+ per-sample column sums, backward)
  {
    const int s = tid >> 8, u = tid & 255;
    const int b = 2 * pair + s;
    const int c4 = u % 12, fg = u / 12;          // 21 frame lanes per channel quad (u < 252)
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    uint16_t* sl = slab + s * (PC_SLAB / 2);
    if (u < 252) {
      for (int f = fg; f < nrows; f += 21) {
        const int frame = f - pad;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (b < B && frame >= 0 && frame < T) {
          const int64_t idx = ((int64_t)b * T + frame) * D + g * PC_G + 4 * c4;
          v = *reinterpret_cast<const float4*>(x + idx);
          if constexpr (BWD) {
            const float4 pr = *reinterpret_cast<const float4*>(pre_in + idx);
            v.x *= b2p_gelu_grad(pr.x);
            v.y *= b2p_gelu_grad(pr.y);
            v.z *= b2p_gelu_grad(pr.z);
            v.w *= b2p_gelu_grad(pr.w);
            cs.x += v.x; cs.y += v.y; cs.z += v.z; cs.w += v.w;
          }
          *reinterpret_cast<uint2*>(side16 + idx) = b2p_pack_bf16x4(v);
        }
        *reinterpret_cast<uint2*>(sl + f * PC_XLD + 4 * c4) = b2p_pack_bf16x4(v);
      }
    }
    if constexpr (BWD) {
      // deterministic column sums: 21 partials per channel quad through LDS (weight buffer 1 is free)
      float* red = reinterpret_cast<float*>(smem + PC_WBUF);
      if (u < 252) *reinterpret_cast<float4*>(red + (s * 21 + fg) * PC_G + 4 * c4) = cs;
      __syncthreads();
      if (u < PC_G && b < B) {
        float acc = 0.f;
        for (int r = 0; r < 21; ++r) acc += red[(s * 21 + r) * PC_G + u];
        colpart[(int64_t)b * D + g * PC_G + u] = acc;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int s = wave >> 2, r0 = 64 * (wave & 3);
  const uint16_t* sl = slab + s * (PC_SLAB / 2);
  const int q = lane >> 4, lr = lane & 15;
  f32x4 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 3; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < PC_NCH; ++ch) {
    if (ch + 1 < PC_NCH) issue_wchunk(wimg, g, ch + 1, smem + ((ch + 1) & 1) * PC_WBUF, wave, lane);
    const char* wbuf = smem + (ch & 1) * PC_WBUF;
#pragma unroll
    for (int kk = 0; kk < PC_TC * PC_G / 32; ++kk) {
      const int kl = kk * 32 + 8 * q;                  // k inside the chunk: tap kl/48, channel kl%48
      const int tapl = kl / PC_G, c = kl - tapl * PC_G;
      bf16x8 a[4], bb[3];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(sl + (r0 + 16 * i + lr + ch * PC_TC + tapl) * PC_XLD + c);
#pragma unroll
      for (int n = 0; n < 3; ++n)
        bb[n] = *reinterpret_cast<const bf16x8*>(wbuf + (16 * n + lr) * (PC_WPR * 16) + (kl >> 3) * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int n = 0; n < 3; ++n) acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[n], acc[i][n], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds rows 4q + r of each 16-row tile, channel lr of each 16-channel tile
  const int b = 2 * pair + s;
  if (b < B) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = r0 + 16 * i + 4 * q + r;
        if (t < T) {
#pragma unroll
          for (int n = 0; n < 3; ++n) {
            const int col = g * PC_G + 16 * n + lr;
            const int64_t idx = ((int64_t)b * T + t) * D + col;
            float v = acc[i][n][r];
            if constexpr (BWD) {
              out[idx] = v + x[idx];
            } else {
              v += bias[col];
              pre_out[idx] = v;
              out[idx] = b2p_gelu(v) + x[idx];
            }
          }
        }
      }
  }
}

// ---- weight gradient. Workgroup (group g, 8 taps tap0 .. tap0+7), 8 waves (wave w: tap tap0+w,
// all 48 x 48 (o, i)); the samples stream through LDS (double-buffered LDS-DMA): the group's dpre
// rows t in [0, 256) and input rows t + tap0 - 64 + [0, 263), both [row][48] bf16. Fragments are
// read k-major (k = t) with ds_read_b64_tr_b16.
constexpr int PW_TAPS = 8;
constexpr int PW_DP = 24 * 1024;               // dpre slab: 256 rows x 96 B
constexpr int PW_E = 32 * 1024;                // input slab: 263 rows x 96 B (<= 32 KB of pieces)
constexpr int PW_BUF = PW_DP + PW_E;
constexpr int PW_LDS = 2 * PW_BUF;             // 112 KB

__device__ __forceinline__ bf16x8 frag_tk(const char* img, int row0, int col0, int kk, int lane) {
  // k-major image [row = k][48 cols] (96-B rows): lane gets column col0 + (lane & 15),
  // k = row0 + 32 kk + 8 (lane >> 4) .. +7 (the MFMA A/B operand layout)
  const int gq = lane >> 4, qq = (lane & 15) >> 2, p = lane & 3;
  s16x4 h[2];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int row = row0 + 32 * kk + 8 * gq + 4 * hh + qq;
    const char* a = img + row * (PC_G * 2) + (col0 + 8 * (p >> 1)) * 2 + 8 * (p & 1);
    h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(a));
  }
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void issue_wsample(const uint16_t* __restrict__ dp16, const uint16_t* __restrict__ e16,
                                              int b, int g, int tap0, int T, int D, char* buf, int wave, int lane) {
  // dpre rows t = 0..255: 6 pieces a row, 1536 pieces = 24 wave-instructions, 3 per wave
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int j = wave * 3 + i;
    const int qp = j * 64 + lane;
    const int t = qp / 6, p = qp - t * 6;
    const void* src = t < T ? (const void*)(dp16 + ((int64_t)b * T + t) * D + g * PC_G + 8 * p) : (const void*)g_pc_zero;
    glds16(src, (lds_t*)(buf + j * 1024));
  }
  // input rows r = 0..262 (frame r + tap0 - 64): 1578 pieces, 32 wave-instructions, 4 per wave
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = wave * 4 + i;
    const int qp = j * 64 + lane;
    const int r = qp / 6, p = qp - r * 6;
    const int frame = r + tap0 - 64;
    const void* src = (r < PC_TMAX + PW_TAPS - 1 && frame >= 0 && frame < T)
                          ? (const void*)(e16 + ((int64_t)b * T + frame) * D + g * PC_G + 8 * p)
                          : (const void*)g_pc_zero;
    glds16(src, (lds_t*)(buf + PW_DP + j * 1024));
  }
}

__global__ void __launch_bounds__(512, 1) pc16_wgrad_k(const uint16_t* __restrict__ dp16,
                                                       const uint16_t* __restrict__ e16, float* __restrict__ dwp,
                                                       int B, int T, int D) {
  __shared__ __attribute__((aligned(1024))) char smem[PW_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NTC = PC_TAPS / PW_TAPS;       // 16 tap chunks per group
  const int lin = xcd_linear(blockIdx.x, gridDim.x);
  const int g = lin / NTC, tap0 = (lin - g * NTC) * PW_TAPS;
  const int nk = (T + 31) / 32;

  f32x4 acc[3][3];
#pragma unroll
  for (int m = 0; m < 3; ++m)
#pragma unroll
    for (int n = 0; n < 3; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_wsample(dp16, e16, 0, g, tap0, T, D, smem, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int b = 0; b < B; ++b) {
    if (b + 1 < B) issue_wsample(dp16, e16, b + 1, g, tap0, T, D, smem + ((b + 1) & 1) * PW_BUF, wave, lane);
    const char* dps = smem + (b & 1) * PW_BUF;
    const char* es = dps + PW_DP;
    for (int kk = 0; kk < nk; ++kk) {
      bf16x8 a[3], bb[3];
#pragma unroll
      for (int m = 0; m < 3; ++m) a[m] = frag_tk(dps, 0, 16 * m, kk, lane);
#pragma unroll
      for (int n = 0; n < 3; ++n) bb[n] = frag_tk(es, wave, 16 * n, kk, lane);
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], bb[n], acc[m][n], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // dwp[g*48 + o][tap*48 + i] (the [O][taps*Ig] layout of b2p_conv_weight_permute)
  const int tap = tap0 + wave;
#pragma unroll
  for (int m = 0; m < 3; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 16 * m + 4 * (lane >> 4) + r;
#pragma unroll
      for (int n = 0; n < 3; ++n)
        dwp[(int64_t)(g * PC_G + o) * PC_KT + tap * PC_G + 16 * n + (lane & 15)] = acc[m][n][r];
    }
}

int pc_check(int64_t B, int64_t T, int64_t D, int64_t groups) {
  B2P_CHECK_ARG(groups > 0 && D == groups * PC_G, "posconv16: needs %d channels per group (D=%lld, groups=%lld)",
                PC_G, (long long)D, (long long)groups);
  B2P_CHECK_ARG(T >= 1 && T <= PC_TMAX, "posconv16: T must be in [1, %d] (T=%lld)", PC_TMAX, (long long)T);
  B2P_CHECK_ARG(B >= 1 && groups * ((B + 1) / 2) < (1ll << 31), "posconv16: bad batch");
  return 0;
}

}  // namespace

extern "C" int b2p_posconv16_fwd(const float* e, const uint16_t* w16, const float* bias, float* xsum, float* pre,
                                 uint16_t* e16, int64_t B, int64_t T, int64_t D, int64_t groups,
                                 b2p_stream_t stream) {
  B2P_CHECK_ARG(e && w16 && bias && xsum && pre && e16, "posconv16_fwd: NULL pointer");
  if (pc_check(B, T, D, groups)) return 1;
  const int npairs = (int)((B + 1) / 2);
  hipLaunchKernelGGL((pc16_k<false>), dim3((unsigned)(groups * npairs)), dim3(512), 0, (hipStream_t)stream, e,
                     (const float*)nullptr, w16, bias, xsum, pre, e16, (float*)nullptr, (int)B, (int)T, (int)D, 64,
                     npairs);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_posconv16_bwd_data(const float* dxsum, const float* pre, const uint16_t* wt16, float* de,
                                      uint16_t* dpre16, float* colpart, int64_t B, int64_t T, int64_t D,
                                      int64_t groups, b2p_stream_t stream) {
  B2P_CHECK_ARG(dxsum && pre && wt16 && de && dpre16 && colpart, "posconv16_bwd_data: NULL pointer");
  if (pc_check(B, T, D, groups)) return 1;
  const int npairs = (int)((B + 1) / 2);
  hipLaunchKernelGGL((pc16_k<true>), dim3((unsigned)(groups * npairs)), dim3(512), 0, (hipStream_t)stream, dxsum,
                     pre, wt16, (const float*)nullptr, de, (float*)nullptr, dpre16, colpart, (int)B, (int)T, (int)D,
                     PC_TAPS - 1 - 64, npairs);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_posconv16_wgrad(const uint16_t* dpre16, const uint16_t* e16, float* dwp, int64_t B, int64_t T,
                                   int64_t D, int64_t groups, b2p_stream_t stream) {
  B2P_CHECK_ARG(dpre16 && e16 && dwp, "posconv16_wgrad: NULL pointer");
  if (pc_check(B, T, D, groups)) return 1;
  hipLaunchKernelGGL(pc16_wgrad_k, dim3((unsigned)(groups * (PC_TAPS / PW_TAPS))), dim3(512), 0,
                     (hipStream_t)stream, dpre16, e16, dwp, (int)B, (int)T, (int)D);
  B2P_CHECK_LAUNCH();
  return 0;
}
