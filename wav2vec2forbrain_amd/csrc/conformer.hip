// Conformer-specific kernels (transformers Wav2Vec2ConformerEncoderLayer / ConvolutionModule /
// RotaryPositionalEmbedding, instantiated by reference
// src/model/w2v_conformer_custom_feat_extractor.py:62-112): rotary embedding, GLU, depthwise
// conv1d (k odd, 'same'), BatchNorm1d training statistics / apply / backward. HBM-bound, fp32,
// channels-last (token-major) like every activation of this library.
#include <initializer_list>
#include <stdlib.h>
#include "common.h"
#include "../../include/b2p_hip.h"

int colsum_impl(const float* X, const float* Y, int64_t batch, int64_t M, int64_t N, int64_t ld, int64_t bstride,
                int mode, float* out, int accumulate, float* part, hipStream_t st);

namespace {
inline unsigned nblk(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }
// q = i / d, r = i - q * d in 32-bit arithmetic when the index space fits (the 64-bit division is a
// ~40-instruction software sequence per thread); `fits` is wave-uniform
__device__ __forceinline__ int64_t div_fit(int64_t i, int64_t d, bool fits) {
  return fits ? (int64_t)((uint32_t)i / (uint32_t)d) : i / d;
}

// x rows (B*T) of H heads x D; cos/sin (T, D). out = x*cos + rotate_half(x)*sin
// rotate_half(x) = cat(-x[D/2:], x[:D/2]); inverse (backward) applies the transpose.
__global__ void rotary_k(const float* __restrict__ x, const float* __restrict__ ct, const float* __restrict__ st,
                         float* __restrict__ out, int64_t rows, int T, int H, int D, int64_t ld, int inverse) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = rows * H * D;
  if (i >= total) return;
  const int d = (int)(i % D);
  const int h = (int)((i / D) % H);
  const int64_t r = i / ((int64_t)D * H);
  const int t = (int)(r % T);
  const float* xr = x + r * ld + (int64_t)h * D;
  const int half = D / 2;
  const float c = ct[(int64_t)t * D + d];
  float v;
  if (!inverse) {
    const float s = st[(int64_t)t * D + d];
    const float rot = d < half ? -xr[d + half] : xr[d - half];
    v = xr[d] * c + rot * s;
  } else {
    // dx[d] = dy[d] cos[d] + (d < half ? dy[d+half] sin[d+half] : -dy[d-half] sin[d-half])
    const float other = d < half ? xr[d + half] * st[(int64_t)t * D + d + half]
                                 : -xr[d - half] * st[(int64_t)t * D + d - half];
    v = xr[d] * c + other;
  }
  out[r * ld + (int64_t)h * D + d] = v;
}

// forward rotation written as a 16-bit GEMM operand (fp16 or bf16), 4 consecutive d per thread
__global__ void rotary16_k(const float* __restrict__ x, const float* __restrict__ ct, const float* __restrict__ st,
                           uint16_t* __restrict__ out, int64_t rows, int T, int H, int D, int64_t ld, int half16) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int D4 = D / 4;
  if (i4 >= rows * H * D4) return;
  const int d = (int)(i4 % D4) * 4;
  const int h = (int)((i4 / D4) % H);
  const int64_t r = i4 / ((int64_t)D4 * H);
  const int t = (int)(r % T);
  const float* xr = x + r * ld + (int64_t)h * D;
  const int half = D / 2;
  const float4 xv = *reinterpret_cast<const float4*>(xr + d);
  const float4 ov = *reinterpret_cast<const float4*>(xr + (d < half ? d + half : d - half));
  const float4 c = *reinterpret_cast<const float4*>(ct + (int64_t)t * D + d);
  const float4 sn = *reinterpret_cast<const float4*>(st + (int64_t)t * D + d);
  const float sg = d < half ? -1.f : 1.f;
  float4 v;
  v.x = xv.x * c.x + sg * ov.x * sn.x;
  v.y = xv.y * c.y + sg * ov.y * sn.y;
  v.z = xv.z * c.z + sg * ov.z * sn.z;
  v.w = xv.w * c.w + sg * ov.w * sn.w;
  *reinterpret_cast<uint2*>(out + r * ld + (int64_t)h * D + d) = b2p_pack16x4(v, half16 != 0);
}

// bf16(dropout(act(pre))): the FFN intermediate recomputed from its fp32 pre-activation for the
// backward weight gradient (the forward GEMM epilogue wrote only the fp16 operand copy); same mask
// index (flat element index) and scale as that epilogue. 4 elements per thread.
__global__ void act_drop_cast16_k(const float* __restrict__ pre, uint16_t* __restrict__ out, int64_t n4, int act,
                                  uint32_t thr, float scale, uint64_t seed, int use_mask,
                                  const uint64_t* __restrict__ epoch) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 >= n4) return;
  seed = b2p_seed_eff(seed, epoch);
  const float4 p = reinterpret_cast<const float4*>(pre)[i4];
  float v[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float a = v[q];
    if (act == B2P_ACT_GELU) a = b2p_gelu(a);
    else if (act == B2P_ACT_SILU) a = b2p_silu(a);
    else if (act == B2P_ACT_SOFTSIGN) a = a / (1.0f + fabsf(a));
    if (use_mask) a = b2p_keep(seed, (uint64_t)(4 * i4 + q), thr) ? a * scale : 0.f;
    v[q] = a;
  }
  reinterpret_cast<uint2*>(out)[i4] = b2p_pack_bf16x4(make_float4(v[0], v[1], v[2], v[3]));
}

// b2p_rotary with 4 consecutive d per thread (D % 8 == 0, 16-B aligned rows): forward and transpose
__global__ void rotary4_k(const float* __restrict__ x, const float* __restrict__ ct, const float* __restrict__ st,
                          float* __restrict__ out, int64_t rows, int T, int H, int D, int64_t ld, int inverse) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int D4 = D / 4;
  if (i4 >= rows * H * D4) return;
  const bool fits = rows * H * D4 < 0x100000000ll;
  const int64_t q4 = div_fit(i4, D4, fits);
  const int d = (int)(i4 - q4 * D4) * 4;
  const int64_t r = div_fit(q4, H, fits);
  const int h = (int)(q4 - r * H);
  const int t = (int)(r - div_fit(r, T, fits) * T);
  const float* xr = x + r * ld + (int64_t)h * D;
  const int half = D / 2;
  const int od = d < half ? d + half : d - half;
  const float4 xv = *reinterpret_cast<const float4*>(xr + d);
  const float4 ov = *reinterpret_cast<const float4*>(xr + od);
  const float4 c = *reinterpret_cast<const float4*>(ct + (int64_t)t * D + d);
  float4 v;
  if (!inverse) {   // x*cos + rotate_half(x)*sin, rotate_half = cat(-x2, x1)
    const float4 sn = *reinterpret_cast<const float4*>(st + (int64_t)t * D + d);
    const float sg = d < half ? -1.f : 1.f;
    v = make_float4(xv.x * c.x + sg * ov.x * sn.x, xv.y * c.y + sg * ov.y * sn.y, xv.z * c.z + sg * ov.z * sn.z,
                    xv.w * c.w + sg * ov.w * sn.w);
  } else {          // dx[d] = dy[d] cos[d] + (d < half ? dy[d+half] sin[d+half] : -dy[d-half] sin[d-half])
    const float4 so = *reinterpret_cast<const float4*>(st + (int64_t)t * D + od);
    const float sg = d < half ? 1.f : -1.f;
    v = make_float4(xv.x * c.x + sg * ov.x * so.x, xv.y * c.y + sg * ov.y * so.y, xv.z * c.z + sg * ov.z * so.z,
                    xv.w * c.w + sg * ov.w * so.w);
  }
  *reinterpret_cast<float4*>(out + r * ld + (int64_t)h * D + d) = v;
}

__global__ void glu_fwd_k(const float* __restrict__ a, float* __restrict__ out, int64_t M, int64_t C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int64_t m = i / C, c = i - m * C;
  const float x = a[m * 2 * C + c], g = a[m * 2 * C + C + c];
  out[i] = x * b2p_sigmoid(g);
}

// glu_fwd_k with 4 channels per thread (C % 4 == 0, 16-B aligned), same expression per element
__global__ void glu_fwd4_k(const float* __restrict__ a, float* __restrict__ out, int64_t M, int64_t C) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t C4 = C / 4;
  if (i4 >= M * C4) return;
  const int64_t m = div_fit(i4, C4, M * C4 < 0x100000000ll), c = (i4 - m * C4) * 4;
  const float4 x = *reinterpret_cast<const float4*>(a + m * 2 * C + c);
  const float4 g = *reinterpret_cast<const float4*>(a + m * 2 * C + C + c);
  *reinterpret_cast<float4*>(out + m * C + c) =
      make_float4(x.x * b2p_sigmoid(g.x), x.y * b2p_sigmoid(g.y), x.z * b2p_sigmoid(g.z), x.w * b2p_sigmoid(g.w));
}

__global__ void glu_bwd_k(const float* __restrict__ a, const float* __restrict__ dout, float* __restrict__ da,
                          int64_t M, int64_t C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int64_t m = i / C, c = i - m * C;
  const float x = a[m * 2 * C + c], g = a[m * 2 * C + C + c];
  const float s = b2p_sigmoid(g);
  const float d = dout[i];
  da[m * 2 * C + c] = d * s;
  da[m * 2 * C + C + c] = d * x * s * (1.f - s);
}

// GLU backward written straight as the bf16 operand of the pointwise-conv-1 backward GEMMs, 4 channels
// per thread (C % 4 == 0): da16[m][c] = bf16(d*s), da16[m][C + c] = bf16(d*x*s*(1-s))
__global__ void glu_bwd16_k(const float* __restrict__ a, const float* __restrict__ dout, uint16_t* __restrict__ da16,
                            int64_t M, int64_t C) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t C4 = C / 4;
  if (i4 >= M * C4) return;
  const int64_t m = div_fit(i4, C4, M * C4 < 0x100000000ll), c = (i4 - m * C4) * 4;
  const float4 x = *reinterpret_cast<const float4*>(a + m * 2 * C + c);
  const float4 g = *reinterpret_cast<const float4*>(a + m * 2 * C + C + c);
  const float4 d = *reinterpret_cast<const float4*>(dout + m * C + c);
  const float s0 = b2p_sigmoid(g.x), s1 = b2p_sigmoid(g.y), s2 = b2p_sigmoid(g.z), s3 = b2p_sigmoid(g.w);
  *reinterpret_cast<uint2*>(da16 + m * 2 * C + c) = b2p_pack_bf16x4(make_float4(d.x * s0, d.y * s1, d.z * s2, d.w * s3));
  *reinterpret_cast<uint2*>(da16 + m * 2 * C + C + c) =
      b2p_pack_bf16x4(make_float4(d.x * x.x * s0 * (1.f - s0), d.y * x.y * s1 * (1.f - s1), d.z * x.z * s2 * (1.f - s2),
                                  d.w * x.w * s3 * (1.f - s3)));
}

// depthwise conv, channels-last, zero 'same' padding p = (K-1)/2: y[b,t,c] = sum_k w[c,k] x[b,t+k-p,c]
__global__ void dwconv_fwd_k(const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y,
                             int64_t B, int64_t T, int64_t C, int K) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T * C) return;
  const int64_t c = i % C, t = (i / C) % T, b = i / (C * T);
  const int p = (K - 1) / 2;
  const float* xb = x + b * T * C + c;
  const float* wc = w + c * K;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    const int64_t s = t + k - p;
    if (s >= 0 && s < T) acc += wc[k] * xb[s * C];
  }
  y[i] = acc;
}

constexpr int DW_TT = 64;   // frame tile of the weight-gradient partials

// LDS-tiled depthwise conv (the Conformer's k31 'same' conv, TF conf ConvolutionModule): a block
// owns 64 channels x 64 frames of one sample; the input frames [t0 - p, t0 + 64 + p) of its channels
// are staged once in LDS (coalesced 256-B rows), every thread keeps its channel's taps in registers
// and a sliding window of 16 + K - 1 frames, and writes 16 outputs (coalesced over channels).
// FLIP: the input-gradient form dx[s] = sum_k w[k] dy[s - k + p] (taps reversed).
constexpr int DWT_T = 64, DW_KMAX = 31;

// rows [s0, s0 + nrows) x 64 channels from c0 of one sample's [T][C] plane into LDS rows of 64
// floats, zero outside [0, T) x [0, C). VEC (C % 4 == 0, 16-B aligned plane): 16 lanes per row with
// float4 loads, every load of the thread issued before its first LDS store (the one-row-per-wave
// scalar staging waited out a load latency per row: the conv kernels ran at ~25 % of HBM speed).
template <bool VEC, int MAXR>
__device__ __forceinline__ void dw_stage(const float* __restrict__ xb, float (*xs)[64], int64_t s0, int nrows,
                                         int64_t T, int64_t C, int64_t c0) {
  if (VEC) {
    constexpr int PASSES = (MAXR + 15) / 16;
    const int lr = threadIdx.x >> 4, lc = (threadIdx.x & 15) * 4;
    const int64_t cc = c0 + lc;
    float4 v[PASSES];
#pragma unroll
    for (int i = 0; i < PASSES; ++i) {
      const int r = lr + 16 * i;
      const int64_t s = s0 + r;
      v[i] = (r < nrows && s >= 0 && s < T && cc < C) ? *reinterpret_cast<const float4*>(xb + s * C + cc)
                                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < PASSES; ++i) {
      const int r = lr + 16 * i;
      if (r < MAXR) *reinterpret_cast<float4*>(&xs[r][lc]) = v[i];
    }
  } else {
    const int cl = threadIdx.x & 63, tg = threadIdx.x >> 6;
    const int64_t c = c0 + cl;
    for (int r = tg; r < MAXR; r += 4) {
      const int64_t s = s0 + r;
      xs[r][cl] = (r < nrows && c < C && s >= 0 && s < T) ? xb[s * C + c] : 0.f;
    }
  }
}

template <bool FLIP, bool VEC>
__global__ void __launch_bounds__(256) dwconv_tile_k(const float* __restrict__ x, const float* __restrict__ w,
                                                     float* __restrict__ y, int64_t T, int64_t C, int K) {
  __shared__ float xs[DWT_T + DW_KMAX - 1][64];
  const int cl = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + cl;
  const int64_t t0 = (int64_t)blockIdx.y * DWT_T;
  const int64_t b = blockIdx.z;
  const int p = (K - 1) / 2;
  const bool cok = c < C;
  dw_stage<VEC, DWT_T + DW_KMAX - 1>(x + b * T * C, xs, t0 - p, DWT_T + K - 1, T, C, (int64_t)blockIdx.x * 64);
  float wr[DW_KMAX];
#pragma unroll
  for (int k = 0; k < DW_KMAX; ++k) wr[k] = (cok && k < K) ? w[c * K + (FLIP ? K - 1 - k : k)] : 0.f;
  __syncthreads();
  constexpr int NO = DWT_T / 4;   // outputs per thread
  float win[NO + DW_KMAX - 1];
#pragma unroll
  for (int j = 0; j < NO + DW_KMAX - 1; ++j) win[j] = (j < NO + K - 1) ? xs[tg * NO + j][cl] : 0.f;
  float* yb = y + b * T * C + c;
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < DW_KMAX; ++k) acc += wr[k] * win[o + k];
    const int64_t t = t0 + tg * NO + o;
    if (cok && t < T) yb[t * C] = acc;
  }
}

// dw partials, LDS-tiled: part[(b*ntile + tile)][k][c] = sum_{t in tile} dy[t][c] x[t + k - p][c]
template <bool VEC>
__global__ void __launch_bounds__(256) dwconv_wgrad_tile_k(const float* __restrict__ x, const float* __restrict__ dy,
                                                           float* __restrict__ part, int64_t T, int64_t C, int K,
                                                           int ntile) {
  __shared__ float xs[DWT_T + DW_KMAX - 1][64];
  __shared__ float ds[DWT_T][64];
  const int cl = threadIdx.x & 63, kg = threadIdx.x >> 6;   // taps 8kg .. 8kg+7
  const int64_t c = (int64_t)blockIdx.x * 64 + cl;
  const int tile = blockIdx.y % ntile;
  const int64_t b = blockIdx.y / ntile;
  const int64_t t0 = (int64_t)tile * DWT_T;
  const int p = (K - 1) / 2;
  const bool cok = c < C;
  dw_stage<VEC, DWT_T + DW_KMAX - 1>(x + b * T * C, xs, t0 - p, DWT_T + K - 1, T, C, (int64_t)blockIdx.x * 64);
  dw_stage<VEC, DWT_T>(dy + b * T * C, ds, t0, DWT_T, T, C, (int64_t)blockIdx.x * 64);
  __syncthreads();
  float acc[8], win[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    acc[q] = 0.f;
    win[q] = xs[kg * 8 + q][cl];
  }
  for (int t = 0; t < DWT_T; ++t) {
    const float g = ds[t][cl];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += g * win[q];
#pragma unroll
    for (int q = 0; q < 7; ++q) win[q] = win[q + 1];
    const int nr = t + 1 + kg * 8 + 7;
    win[7] = nr < DWT_T + DW_KMAX - 1 ? xs[nr][cl] : 0.f;
  }
  if (cok) {
    float* pp = part + (int64_t)blockIdx.y * K * C;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = kg * 8 + q;
      if (k < K) pp[(int64_t)k * C + c] = acc[q];
    }
  }
}

__global__ void dw_transpose_k(const float* __restrict__ kc, float* __restrict__ ck, int64_t C, int K) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * K) return;
  const int64_t c = i / K, k = i % K;
  ck[i] = kc[k * C + c];
}

// ---- BatchNorm1d (training statistics over M rows, per channel)
__global__ void bn_finalize_k(const float* __restrict__ sum, const float* __restrict__ sqdev, const float* __restrict__ mean,
                              float* __restrict__ rstd, float* __restrict__ run_mean, float* __restrict__ run_var,
                              int64_t C, int64_t count, float eps, float momentum, const int32_t* __restrict__ gate,
                              int64_t* __restrict__ nbt = nullptr) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mu = mean[c];
  const float var = sqdev[c] / (float)count;
  rstd[c] = rsqrtf(var + eps);
  // LayerDrop: a replay that skips this layer leaves the running statistics untouched (the reference
  // never runs the layer), so the captured step needs no snapshot / restore of them
  if (b2p_gated_off(gate)) return;
  if (nbt && c == 0) *nbt += 1;   // BatchNorm's num_batches_tracked (torch _BatchNorm.forward, training)
  if (run_mean) run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
  if (run_var) {
    const float unb = count > 1 ? sqdev[c] / (float)(count - 1) : var;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
  (void)sum;
}

__global__ void scale_k(float* __restrict__ v, int64_t n, float s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] *= s;
}

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == B2P_ACT_SILU) return b2p_silu(v);
  if (act == B2P_ACT_GELU) return b2p_gelu(v);
  return v;
}
__device__ __forceinline__ float act_g(float v, int act) {
  if (act == B2P_ACT_SILU) return b2p_silu_grad(v);
  if (act == B2P_ACT_GELU) return b2p_gelu_grad(v);
  return 1.f;
}

// y = act(pre), pre = (x - mean) * rstd * gamma + beta
__global__ void bn_apply_k(const float* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ rstd,
                           const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ y,
                           float* __restrict__ pre, int64_t M, int64_t C, int act) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int64_t c = i % C;
  const float v = (x[i] - mean[c]) * rstd[c] * gamma[c] + beta[c];
  if (pre) pre[i] = v;
  y[i] = act_f(v, act);
}

// g = dy * act'(pre)  (written to g)
__global__ void bn_grad_pre_k(const float* __restrict__ dy, const float* __restrict__ pre, float* __restrict__ g,
                              int64_t n, int act) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  g[i] = dy[i] * act_g(pre[i], act);
}

// dx = gamma*rstd/M * (M*g - sum_g - xhat * sum_gxhat), xhat = (x-mean)*rstd
__global__ void bn_bwd_dx_k(const float* __restrict__ g, const float* __restrict__ x, const float* __restrict__ mean,
                            const float* __restrict__ rstd, const float* __restrict__ gamma,
                            const float* __restrict__ sum_g, const float* __restrict__ sum_gx, float* __restrict__ dx,
                            int64_t M, int64_t C, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int64_t c = i % C;
  const float xh = (x[i] - mean[c]) * rstd[c];
  const float inv = 1.f / (float)count;
  dx[i] = gamma[c] * rstd[c] * (g[i] - sum_g[c] * inv - xh * sum_gx[c] * inv);
}

// xhat products for dgamma: t = g * (x - mean) * rstd
__global__ void bn_gxhat_k(const float* __restrict__ g, const float* __restrict__ x, const float* __restrict__ mean,
                           const float* __restrict__ rstd, float* __restrict__ t, int64_t M, int64_t C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int64_t c = i % C;
  t[i] = g[i] * (x[i] - mean[c]) * rstd[c];
}

// channel group of float4 element i: a 32-bit modulo when the tensor allows (the 64-bit one is a ~40-
// instruction software sequence, the largest VALU cost of these byte-bound passes); wave-uniform branch
__device__ __forceinline__ int64_t chan4(int64_t i, int64_t n4, int64_t C4) {
  return n4 < 0x100000000ll ? (int64_t)((uint32_t)i % (uint32_t)C4) : i % C4;
}
// float4 forms of the four BatchNorm elementwise passes above (C % 4 == 0, 16-B aligned tensors):
// the same per-element expressions, 4 consecutive channels per thread, one index division per 4
// elements (the scalar kernels' 64-bit modulo per element held them at ~60 % of HBM speed)
// y (fp32), y16 (fp16 when half, else bf16) and y16b (bf16) are each optional: the Conformer conv module
// keeps only the 16-bit operands of the pointwise conv 2 (its forward GEMM and its weight gradient)
__global__ void bn_apply4_k(const float4* __restrict__ x, const float* __restrict__ mean, const float* __restrict__ rstd,
                            const float* __restrict__ gamma, const float* __restrict__ beta, float4* __restrict__ y,
                            float4* __restrict__ pre, int64_t n4, int64_t C4, int act, uint2* __restrict__ y16 = nullptr,
                            int half = 0, uint2* __restrict__ y16b = nullptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int64_t c = 4 * chan4(i, n4, C4);
  const float4 xv = x[i];
  const float* xp = reinterpret_cast<const float*>(&xv);
  float v[4], o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = (xp[q] - mean[c + q]) * rstd[c + q] * gamma[c + q] + beta[c + q];
    o[q] = act_f(v[q], act);
  }
  if (pre) pre[i] = make_float4(v[0], v[1], v[2], v[3]);
  const float4 ov = make_float4(o[0], o[1], o[2], o[3]);
  if (y) y[i] = ov;
  if (y16) y16[i] = b2p_pack16x4(ov, half != 0);
  if (y16b) y16b[i] = b2p_pack_bf16x4(ov);
}

__global__ void bn_grad_pre4_k(const float4* __restrict__ dy, const float4* __restrict__ pre, float4* __restrict__ g,
                               int64_t n4, int act) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 d = dy[i], p = pre[i];
  g[i] = make_float4(d.x * act_g(p.x, act), d.y * act_g(p.y, act), d.z * act_g(p.z, act), d.w * act_g(p.w, act));
}

__global__ void bn_bwd_dx4_k(const float4* __restrict__ g, const float4* __restrict__ x, const float* __restrict__ mean,
                             const float* __restrict__ rstd, const float* __restrict__ gamma,
                             const float* __restrict__ sum_g, const float* __restrict__ sum_gx, float4* __restrict__ dx,
                             int64_t n4, int64_t C4, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int64_t c = 4 * chan4(i, n4, C4);
  const float4 gv = g[i], xv = x[i];
  const float* gp = reinterpret_cast<const float*>(&gv);
  const float* xp = reinterpret_cast<const float*>(&xv);
  const float inv = 1.f / (float)count;
  float o[4];
  // the scalar kernel's operation sequence spelled out (its contraction: g - inv * sum_g as one fma, the
  // rest rounded per operation), so both forms write the same bits
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma clang fp contract(off)
    const float xh = (xp[q] - mean[c + q]) * rstd[c + q];
    const float t = __builtin_fmaf(-inv, sum_g[c + q], gp[q]);
    const float u = inv * (xh * sum_gx[c + q]);
    o[q] = (gamma[c + q] * rstd[c + q]) * (t - u);
  }
  dx[i] = make_float4(o[0], o[1], o[2], o[3]);
}

__global__ void bn_gxhat4_k(const float4* __restrict__ g, const float4* __restrict__ x, const float* __restrict__ mean,
                            const float* __restrict__ rstd, float4* __restrict__ t, int64_t n4, int64_t C4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int64_t c = 4 * chan4(i, n4, C4);
  const float4 gv = g[i], xv = x[i];
  const float* gp = reinterpret_cast<const float*>(&gv);
  const float* xp = reinterpret_cast<const float*>(&xv);
  float o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = gp[q] * (xp[q] - mean[c + q]) * rstd[c + q];
  t[i] = make_float4(o[0], o[1], o[2], o[3]);
}

__global__ void dropout_scale_k(const float* __restrict__ x, float* __restrict__ y, int64_t n, uint32_t thr,
                                float scale, uint64_t seed, int use_mask, const uint64_t* __restrict__ epoch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  seed = b2p_seed_eff(seed, epoch);
  y[i] = (!use_mask || b2p_keep(seed, (uint64_t)i, thr)) ? x[i] * scale : 0.f;
}

constexpr int DCC_ROWS = 64;   // rows per block (~1000 blocks over an 8k x 1024 tensor: enough loads in flight)
// y16 = bf16(mask(x) * scale) over an M x N row-major tensor (N % 4 == 0, 16-B aligned rows), plus
// optional per-DCC_ROWS-row column partial sums of the fp32 values, part[blk][n] (the bias gradient of
// the Linear that produced x; b2p_colsum_parts finishes it): the output-dropout backward of a
// Conformer block (dropout, its bf16 GEMM operand and its bias gradient in one pass over dy).
// Grid (ceil(N/128), ceil(M/DCC_ROWS)); 32 float4 columns x 8 row lanes per block; mask index = m*N + n,
// the element index dropout_scale_k and the forward GEMM epilogue use.
__global__ void __launch_bounds__(256) drop_cast_colsum_k(const float* __restrict__ x, uint16_t* __restrict__ y16,
                                                          float* __restrict__ part, int64_t M, int64_t N, uint32_t thr,
                                                          float scale, uint64_t seed, int use_mask,
                                                          const uint64_t* __restrict__ epoch) {
  __shared__ float4 red[8][32];
  const int c4 = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int64_t n = (int64_t)blockIdx.x * 128 + 4 * c4;
  const int64_t m0 = (int64_t)blockIdx.y * DCC_ROWS;
  const int64_t m1 = m0 + DCC_ROWS < M ? m0 + DCC_ROWS : M;
  seed = b2p_seed_eff(seed, epoch);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
#pragma unroll 4
    for (int64_t m = m0 + rl; m < m1; m += 8) {
      const int64_t i = m * N + n;
      float4 v = *reinterpret_cast<const float4*>(x + i);
      v.x *= scale; v.y *= scale; v.z *= scale; v.w *= scale;
      if (use_mask) {
        bool k[4];
        b2p_keep4(seed, (uint64_t)i, thr, k);   // i % 4 == 0
        if (!k[0]) v.x = 0.f;
        if (!k[1]) v.y = 0.f;
        if (!k[2]) v.z = 0.f;
        if (!k[3]) v.w = 0.f;
      }
      *reinterpret_cast<uint2*>(y16 + i) = b2p_pack_bf16x4(v);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  if (!part) return;
  red[rl][c4] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float4 t = red[0][c4];
#pragma unroll
    for (int r = 1; r < 8; ++r) {
      const float4 u = red[r][c4];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    *reinterpret_cast<float4*>(part + (int64_t)blockIdx.y * N + n) = t;
  }
}
}  // namespace

extern "C" int b2p_rotary(const float* x, const float* cos_t, const float* sin_t, float* out, int64_t B, int64_t T,
                          int64_t H, int64_t D, int64_t ld, int inverse, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && cos_t && sin_t && out && x != out, "rotary: bad pointers");
  B2P_CHECK_ARG(D % 2 == 0, "rotary: head dim must be even");
  const int64_t n = B * T * H * D;
  if (n <= 0) return 0;
  if (D % 8 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15u) == 0 && ((uintptr_t)out & 15u) == 0)
    hipLaunchKernelGGL(rotary4_k, dim3(nblk(n / 4)), dim3(256), 0, (hipStream_t)stream, x, cos_t, sin_t, out, B * T,
                       (int)T, (int)H, (int)D, ld, inverse);
  else
    hipLaunchKernelGGL(rotary_k, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, x, cos_t, sin_t, out, B * T,
                       (int)T, (int)H, (int)D, ld, inverse);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_glu_fwd(const float* a, float* out, int64_t M, int64_t C, b2p_stream_t stream) {
  B2P_CHECK_ARG(a && out, "glu_fwd: NULL");
  if (M * C <= 0) return 0;
  if (C % 4 == 0 && ((uintptr_t)a & 15u) == 0 && ((uintptr_t)out & 15u) == 0)
    hipLaunchKernelGGL(glu_fwd4_k, dim3(nblk(M * C / 4)), dim3(256), 0, (hipStream_t)stream, a, out, M, C);
  else
    hipLaunchKernelGGL(glu_fwd_k, dim3(nblk(M * C)), dim3(256), 0, (hipStream_t)stream, a, out, M, C);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_glu_bwd(const float* a, const float* dout, float* da, int64_t M, int64_t C, b2p_stream_t stream) {
  B2P_CHECK_ARG(a && dout && da, "glu_bwd: NULL");
  if (M * C <= 0) return 0;
  hipLaunchKernelGGL(glu_bwd_k, dim3(nblk(M * C)), dim3(256), 0, (hipStream_t)stream, a, dout, da, M, C);
  B2P_CHECK_LAUNCH();
  return 0;
}

static bool dw_vec_ok(const float* p, int64_t C) { return C % 4 == 0 && ((uintptr_t)p & 15u) == 0; }

extern "C" int b2p_dwconv_fwd(const float* x, const float* w, float* y, int64_t B, int64_t T, int64_t C, int K,
                              b2p_stream_t stream) {
  B2P_CHECK_ARG(x && w && y, "dwconv_fwd: NULL");
  B2P_CHECK_ARG(K % 2 == 1, "dwconv: kernel size must be odd ('same' padding)");
  const int64_t n = B * T * C;
  if (n <= 0) return 0;
  const bool vec = dw_vec_ok(x, C);
  if (K <= DW_KMAX)
    hipLaunchKernelGGL((vec ? dwconv_tile_k<false, true> : dwconv_tile_k<false, false>),
                       dim3((unsigned)((C + 63) / 64), (unsigned)((T + DWT_T - 1) / DWT_T), (unsigned)B), dim3(256), 0,
                       (hipStream_t)stream, x, w, y, T, C, K);
  else
    hipLaunchKernelGGL(dwconv_fwd_k, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, x, w, y, B, T, C, K);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t b2p_dwconv_bwd_workspace(int64_t B, int64_t T, int64_t C, int K) {
  const int64_t ntile = (T + DW_TT - 1) / DW_TT;
  const int64_t rows = B * ntile;
  return rows * K * C + (int64_t)K * C + ((rows + 255) / 256) * K * C;
}

extern "C" int b2p_dwconv_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw, int64_t B,
                              int64_t T, int64_t C, int K, float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && w && dy && workspace, "dwconv_bwd: NULL");
  B2P_CHECK_ARG(K % 2 == 1 && K <= 32, "dwconv_bwd: odd kernel size <= 31 supported");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = B * T * C;
  if (n <= 0) return 0;
  const bool vec = dw_vec_ok(x, C) && dw_vec_ok(dy, C);
  if (dx)
    hipLaunchKernelGGL((vec ? dwconv_tile_k<true, true> : dwconv_tile_k<true, false>),
                       dim3((unsigned)((C + 63) / 64), (unsigned)((T + DWT_T - 1) / DWT_T), (unsigned)B), dim3(256), 0,
                       st, dy, w, dx, T, C, K);
  if (dw) {
    const int ntile = (int)((T + DW_TT - 1) / DW_TT);
    float* part = workspace;
    float* kc = part + B * ntile * (int64_t)K * C;
    float* p2 = kc + (int64_t)K * C;
    hipLaunchKernelGGL(vec ? dwconv_wgrad_tile_k<true> : dwconv_wgrad_tile_k<false>,
                       dim3((unsigned)((C + 63) / 64), (unsigned)(B * ntile)), dim3(256), 0, st, x, dy, part, T, C, K,
                       ntile);
    if (colsum_impl(part, nullptr, 1, B * ntile, (int64_t)K * C, (int64_t)K * C, 0, 0, kc, 0, p2, st)) return 1;
    hipLaunchKernelGGL(dw_transpose_k, dim3(nblk(C * K)), dim3(256), 0, st, kc, dw, C, K);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t b2p_batchnorm_workspace(int64_t M, int64_t C) {
  return M * C + 4 * C + ((M + 255) / 256) * C;
}

// training-mode BN forward: mean/rstd (saved), running stats update, y = act(BN(x)), pre saved
static bool bn_vec(int64_t C, std::initializer_list<const void*> ps) {
  if (C % 4 != 0) return false;
  for (const void* p : ps)
    if (p && ((uintptr_t)p & 15u) != 0) return false;
  return true;
}
static void bn_apply_launch(const float* x, const float* mean, const float* rstd, const float* gamma, const float* beta,
                            float* y, float* pre, int64_t M, int64_t C, int act, hipStream_t st) {
  if (bn_vec(C, {x, y, pre}))
    hipLaunchKernelGGL(bn_apply4_k, dim3(nblk(M * C / 4)), dim3(256), 0, st, reinterpret_cast<const float4*>(x), mean,
                       rstd, gamma, beta, reinterpret_cast<float4*>(y), reinterpret_cast<float4*>(pre), M * C / 4, C / 4,
                       act, (uint2*)nullptr, 0, (uint2*)nullptr);
  else
    hipLaunchKernelGGL(bn_apply_k, dim3(nblk(M * C)), dim3(256), 0, st, x, mean, rstd, gamma, beta, y, pre, M, C, act);
}
// the 16-bit-output form (vector path only: C % 4 == 0, 16-B aligned fp32 and 8-B aligned 16-bit pointers,
// checked by the callers)
static void bn_apply16_launch(const float* x, const float* mean, const float* rstd, const float* gamma,
                              const float* beta, float* y, uint16_t* y16, int half, uint16_t* y16b, float* pre, int64_t M,
                              int64_t C, int act, hipStream_t st) {
  hipLaunchKernelGGL(bn_apply4_k, dim3(nblk(M * C / 4)), dim3(256), 0, st, reinterpret_cast<const float4*>(x), mean,
                     rstd, gamma, beta, reinterpret_cast<float4*>(y), reinterpret_cast<float4*>(pre), M * C / 4, C / 4,
                     act, reinterpret_cast<uint2*>(y16), half, reinterpret_cast<uint2*>(y16b));
}
bool bn16_ok(int64_t C, const void* x, const void* y, const void* pre, const void* y16, const void* y16b) {
  return bn_vec(C, {x, y, pre}) && ((uintptr_t)y16 & 7u) == 0 && ((uintptr_t)y16b & 7u) == 0;
}
static void bn_grad_pre_launch(const float* dy, const float* pre, float* g, int64_t M, int64_t C, int act,
                               hipStream_t st) {
  if (bn_vec(C, {dy, pre, g}))
    hipLaunchKernelGGL(bn_grad_pre4_k, dim3(nblk(M * C / 4)), dim3(256), 0, st, reinterpret_cast<const float4*>(dy),
                       reinterpret_cast<const float4*>(pre), reinterpret_cast<float4*>(g), M * C / 4, act);
  else
    hipLaunchKernelGGL(bn_grad_pre_k, dim3(nblk(M * C)), dim3(256), 0, st, dy, pre, g, M * C, act);
}
static void bn_gxhat_launch(const float* g, const float* x, const float* mean, const float* rstd, float* t, int64_t M,
                            int64_t C, hipStream_t st) {
  if (bn_vec(C, {g, x, t}))
    hipLaunchKernelGGL(bn_gxhat4_k, dim3(nblk(M * C / 4)), dim3(256), 0, st, reinterpret_cast<const float4*>(g),
                       reinterpret_cast<const float4*>(x), mean, rstd, reinterpret_cast<float4*>(t), M * C / 4, C / 4);
  else
    hipLaunchKernelGGL(bn_gxhat_k, dim3(nblk(M * C)), dim3(256), 0, st, g, x, mean, rstd, t, M, C);
}
static void bn_bwd_dx_launch(const float* g, const float* x, const float* mean, const float* rstd, const float* gamma,
                             const float* sum_g, const float* sum_gx, float* dx, int64_t M, int64_t C, int64_t count,
                             hipStream_t st) {
  // the float4 form spells out the scalar form's contraction (bitwise equal:
  // tests/test_kernels_gpu.py::test_conv_module_vector_paths_bitwise_equal_scalar_paths); B2P_BN_DX4=0: scalar
  static const bool dx4 = !getenv("B2P_BN_DX4") || atoi(getenv("B2P_BN_DX4")) != 0;
  if (dx4 && bn_vec(C, {g, x, dx}))
    hipLaunchKernelGGL(bn_bwd_dx4_k, dim3(nblk(M * C / 4)), dim3(256), 0, st, reinterpret_cast<const float4*>(g),
                       reinterpret_cast<const float4*>(x), mean, rstd, gamma, sum_g, sum_gx, reinterpret_cast<float4*>(dx),
                       M * C / 4, C / 4, count);
  else
    hipLaunchKernelGGL(bn_bwd_dx_k, dim3(nblk(M * C)), dim3(256), 0, st, g, x, mean, rstd, gamma, sum_g, sum_gx, dx, M,
                       C, count);
}

namespace {
// num_batches_tracked of the next training BatchNorm's statistics launch (b2p_batchnorm_count_next),
// incremented by bn_finalize_k under the LayerDrop gate; consumed by that launch
thread_local int64_t* g_bn_counter = nullptr;
int64_t* take_bn_counter() {
  int64_t* p = g_bn_counter;
  g_bn_counter = nullptr;
  return p;
}
}  // namespace

extern "C" int b2p_batchnorm_count_next(int64_t* num_batches_tracked) {
  g_bn_counter = num_batches_tracked;
  return 0;
}

extern "C" int b2p_batchnorm_fwd(const float* x, const float* gamma, const float* beta, float* running_mean,
                                 float* running_var, float* y, float* pre, float* mean, float* rstd, int64_t M,
                                 int64_t C, float eps, float momentum, int act, float* workspace,
                                 b2p_stream_t stream) {
  int64_t* nbt = take_bn_counter();
  B2P_CHECK_ARG(x && gamma && beta && y && mean && rstd && workspace, "batchnorm_fwd: NULL");
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0) return 0;
  float* sqdev = workspace;
  float* part = workspace + 4 * C;
  // two-pass statistics: mean, then sum of squared deviations (mode 3)
  if (colsum_impl(x, nullptr, 1, M, C, C, 0, 0, mean, 0, part, st)) return 1;
  hipLaunchKernelGGL(scale_k, dim3(nblk(C)), dim3(256), 0, st, mean, C, 1.f / (float)M);
  if (colsum_impl(x, mean, 1, M, C, C, 0, 3, sqdev, 0, part, st)) return 1;
  hipLaunchKernelGGL(bn_finalize_k, dim3(nblk(C)), dim3(256), 0, st, (const float*)nullptr, sqdev, mean, rstd,
                     running_mean, running_var, C, M, eps, momentum, b2p_gate(), nbt);
  bn_apply_launch(x, mean, rstd, gamma, beta, y, pre, M, C, act, st);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_batchnorm_fwd16(const float* x, const float* gamma, const float* beta, float* running_mean,
                                   float* running_var, float* y, uint16_t* y16, int y16_fp16, uint16_t* y16b, float* pre,
                                   float* mean, float* rstd, int64_t M, int64_t C, float eps, float momentum, int act,
                                   float* workspace, b2p_stream_t stream) {
  int64_t* nbt = take_bn_counter();
  B2P_CHECK_ARG(x && gamma && beta && (y || y16 || y16b) && mean && rstd && workspace, "batchnorm_fwd16: NULL");
  B2P_CHECK_ARG(bn16_ok(C, x, y, pre, y16, y16b), "batchnorm_fwd16: needs C %% 4 == 0 and aligned pointers");
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0) return 0;
  float* sqdev = workspace;
  float* part = workspace + 4 * C;
  if (colsum_impl(x, nullptr, 1, M, C, C, 0, 0, mean, 0, part, st)) return 1;
  hipLaunchKernelGGL(scale_k, dim3(nblk(C)), dim3(256), 0, st, mean, C, 1.f / (float)M);
  if (colsum_impl(x, mean, 1, M, C, C, 0, 3, sqdev, 0, part, st)) return 1;
  hipLaunchKernelGGL(bn_finalize_k, dim3(nblk(C)), dim3(256), 0, st, (const float*)nullptr, sqdev, mean, rstd,
                     running_mean, running_var, C, M, eps, momentum, b2p_gate(), nbt);
  bn_apply16_launch(x, mean, rstd, gamma, beta, y, y16, y16_fp16, y16b, pre, M, C, act, st);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_batchnorm_apply16(const float* x, const float* mean, const float* rstd, const float* gamma,
                                     const float* beta, float* y, uint16_t* y16, int y16_fp16, uint16_t* y16b, float* pre,
                                     int64_t M, int64_t C, int act, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && mean && rstd && gamma && beta && (y || y16 || y16b), "batchnorm_apply16: NULL");
  B2P_CHECK_ARG(bn16_ok(C, x, y, pre, y16, y16b), "batchnorm_apply16: needs C %% 4 == 0 and aligned pointers");
  if (M * C <= 0) return 0;
  bn_apply16_launch(x, mean, rstd, gamma, beta, y, y16, y16_fp16, y16b, pre, M, C, act, (hipStream_t)stream);
  B2P_CHECK_LAUNCH();
  return 0;
}

// eval-mode BN (running statistics) — forward only
extern "C" int b2p_batchnorm_eval(const float* x, const float* gamma, const float* beta, const float* running_mean,
                                  const float* running_var, float* y, int64_t M, int64_t C, float eps, int act,
                                  float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && gamma && beta && running_mean && running_var && y && workspace, "batchnorm_eval: NULL");
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0) return 0;
  float* rstd = workspace;
  float* sq = workspace + C;
  B2P_CHECK_HIP(hipMemcpyAsync(sq, running_var, C * sizeof(float), hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(bn_finalize_k, dim3(nblk(C)), dim3(256), 0, st, (const float*)nullptr, sq, running_mean, rstd,
                     (float*)nullptr, (float*)nullptr, C, (int64_t)1, eps, 0.f, (const int32_t*)nullptr);
  bn_apply_launch(x, running_mean, rstd, gamma, beta, y, nullptr, M, C, act, st);
  B2P_CHECK_LAUNCH();
  return 0;
}

// BN backward through the fused activation: dy (grad of act output) -> dx, dgamma, dbeta
extern "C" int b2p_batchnorm_bwd(const float* dy, const float* pre, const float* x, const float* mean,
                                 const float* rstd, const float* gamma, float* dx, float* dgamma, float* dbeta,
                                 int64_t M, int64_t C, int act, float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(dy && pre && x && mean && rstd && gamma && dx && dgamma && dbeta && workspace, "batchnorm_bwd: NULL");
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0) return 0;
  float* g = workspace;                 // M*C
  float* part = workspace + M * C + 4 * C;
  bn_grad_pre_launch(dy, pre, g, M, C, act, st);
  if (colsum_impl(g, nullptr, 1, M, C, C, 0, 0, dbeta, 0, part, st)) return 1;
  bn_gxhat_launch(g, x, mean, rstd, dx, M, C, st);
  if (colsum_impl(dx, nullptr, 1, M, C, C, 0, 0, dgamma, 0, part, st)) return 1;
  bn_bwd_dx_launch(g, x, mean, rstd, gamma, dbeta, dgamma, dx, M, C, M, st);
  B2P_CHECK_LAUNCH();
  return 0;
}

// ---- staged BatchNorm (SyncBN: the caller all-reduces the per-channel sums between stages)
extern "C" int b2p_batchnorm_stats(const float* x, const float* center, float* out, int64_t M, int64_t C,
                                   float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && out && workspace, "batchnorm_stats: NULL");
  if (M <= 0 || C <= 0) return 0;
  return colsum_impl(x, center, 1, M, C, C, 0, center ? 3 : 0, out, 0, workspace + 4 * C, (hipStream_t)stream);
}

extern "C" int b2p_batchnorm_finalize(float* sum_or_mean, const float* sqdev, float* rstd, float* running_mean,
                                      float* running_var, int64_t C, int64_t count, float eps, float momentum,
                                      int phase, b2p_stream_t stream) {
  int64_t* nbt = phase == 1 ? take_bn_counter() : nullptr;
  B2P_CHECK_ARG(sum_or_mean && count > 0, "batchnorm_finalize: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (C <= 0) return 0;
  if (phase == 0) {
    hipLaunchKernelGGL(scale_k, dim3(nblk(C)), dim3(256), 0, st, sum_or_mean, C, 1.f / (float)count);
  } else {
    B2P_CHECK_ARG(sqdev && rstd, "batchnorm_finalize: phase 1 needs sqdev and rstd");
    hipLaunchKernelGGL(bn_finalize_k, dim3(nblk(C)), dim3(256), 0, st, (const float*)nullptr, sqdev,
                       (const float*)sum_or_mean, rstd, running_mean, running_var, C, count, eps, momentum,
                       b2p_gate(), nbt);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_batchnorm_apply(const float* x, const float* mean, const float* rstd, const float* gamma,
                                   const float* beta, float* y, float* pre, int64_t M, int64_t C, int act,
                                   b2p_stream_t stream) {
  B2P_CHECK_ARG(x && mean && rstd && gamma && beta && y, "batchnorm_apply: NULL");
  if (M * C <= 0) return 0;
  bn_apply_launch(x, mean, rstd, gamma, beta, y, pre, M, C, act, (hipStream_t)stream);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_batchnorm_bwd_sums(const float* dy, const float* pre, const float* x, const float* mean,
                                      const float* rstd, float* g, float* sum_g, float* sum_gx, int64_t M, int64_t C,
                                      int act, float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(dy && pre && x && mean && rstd && g && sum_g && sum_gx && workspace, "batchnorm_bwd_sums: NULL");
  hipStream_t st = (hipStream_t)stream;
  if (M <= 0) return 0;
  float* t = workspace;                  // M*C: g * xhat
  float* part = workspace + M * C + 4 * C;
  bn_grad_pre_launch(dy, pre, g, M, C, act, st);
  if (colsum_impl(g, nullptr, 1, M, C, C, 0, 0, sum_g, 0, part, st)) return 1;
  bn_gxhat_launch(g, x, mean, rstd, t, M, C, st);
  if (colsum_impl(t, nullptr, 1, M, C, C, 0, 0, sum_gx, 0, part, st)) return 1;
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_batchnorm_bwd_dx(const float* g, const float* x, const float* mean, const float* rstd,
                                    const float* gamma, const float* sum_g, const float* sum_gx, float* dx, int64_t M,
                                    int64_t C, int64_t count, b2p_stream_t stream) {
  B2P_CHECK_ARG(g && x && mean && rstd && gamma && sum_g && sum_gx && dx && count > 0, "batchnorm_bwd_dx: bad args");
  if (M * C <= 0) return 0;
  bn_bwd_dx_launch(g, x, mean, rstd, gamma, sum_g, sum_gx, dx, M, C, count, (hipStream_t)stream);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_dropout_scaled(const float* x, float* y, int64_t n, float p, uint64_t seed, float scale,
                                  b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "dropout_scaled: NULL");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "dropout_scaled: p in [0,1)");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dropout_scale_k, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, x, y, n,
                     b2p_dropout_threshold(p), p > 0.f ? scale / (1.f - p) : scale, seed, p > 0.f ? 1 : 0,
                     b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t b2p_drop_cast_colsum_parts(int64_t M) { return M > 0 ? (M + DCC_ROWS - 1) / DCC_ROWS : 0; }

extern "C" int b2p_drop_cast_colsum(const float* x, uint16_t* y16, float* part, int64_t M, int64_t N, float p,
                                    uint64_t seed, float scale, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y16, "drop_cast_colsum: NULL");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "drop_cast_colsum: p in [0,1)");
  B2P_CHECK_ARG(N % 4 == 0 && ((uintptr_t)x & 15u) == 0 && ((uintptr_t)y16 & 7u) == 0 &&
                    ((uintptr_t)part & 15u) == 0,
                "drop_cast_colsum: needs N % 4 == 0, 16-B aligned x / part, 8-B aligned y16");
  if (M <= 0 || N <= 0) return 0;
  const dim3 grid((unsigned)((N + 127) / 128), (unsigned)((M + DCC_ROWS - 1) / DCC_ROWS));
  hipLaunchKernelGGL(drop_cast_colsum_k, grid, dim3(256), 0, (hipStream_t)stream, x, y16, part, M, N,
                     b2p_dropout_threshold(p), p > 0.f ? scale / (1.f - p) : scale, seed, p > 0.f ? 1 : 0,
                     b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_rotary16(const float* x, const float* cos_t, const float* sin_t, uint16_t* out, int fp16, int64_t B,
                            int64_t T, int64_t H, int64_t D, int64_t ld, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && cos_t && sin_t && out, "rotary16: NULL pointer");
  B2P_CHECK_ARG(D % 8 == 0 && ld % 4 == 0 && ((uintptr_t)x & 15u) == 0 && ((uintptr_t)out & 7u) == 0,
                "rotary16: head dim must be a multiple of 8 and rows 16-B aligned");
  const int64_t n4 = B * T * H * (D / 4);
  if (n4 <= 0) return 0;
  hipLaunchKernelGGL(rotary16_k, dim3(nblk(n4)), dim3(256), 0, (hipStream_t)stream, x, cos_t, sin_t, out, B * T,
                     (int)T, (int)H, (int)D, ld, fp16);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_act_dropout_cast16(const float* pre, uint16_t* out, int64_t n, int act, float p, uint64_t seed,
                                      b2p_stream_t stream) {
  B2P_CHECK_ARG(pre && out, "act_dropout_cast16: NULL pointer");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "act_dropout_cast16: p in [0,1)");
  B2P_CHECK_ARG(n % 4 == 0 && ((uintptr_t)pre & 15u) == 0 && ((uintptr_t)out & 7u) == 0,
                "act_dropout_cast16: n % 4 == 0 and aligned pointers required");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(act_drop_cast16_k, dim3(nblk(n / 4)), dim3(256), 0, (hipStream_t)stream, pre, out, n / 4, act,
                     b2p_dropout_threshold(p), p > 0.f ? 1.f / (1.f - p) : 1.f, seed, p > 0.f ? 1 : 0,
                     b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_glu_bwd16(const float* a, const float* dout, uint16_t* da16, int64_t M, int64_t C,
                             b2p_stream_t stream) {
  B2P_CHECK_ARG(a && dout && da16, "glu_bwd16: NULL pointer");
  B2P_CHECK_ARG(C % 4 == 0 && ((uintptr_t)a & 15u) == 0 && ((uintptr_t)dout & 15u) == 0 && ((uintptr_t)da16 & 7u) == 0,
                "glu_bwd16: needs C %% 4 == 0 and aligned pointers");
  if (M * C <= 0) return 0;
  hipLaunchKernelGGL(glu_bwd16_k, dim3(nblk(M * C / 4)), dim3(256), 0, (hipStream_t)stream, a, dout, da16, M, C);
  B2P_CHECK_LAUNCH();
  return 0;
}
