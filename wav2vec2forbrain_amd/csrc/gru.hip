// Bidirectional GRU recurrence (nn.GRU semantics, gate order r, z, n) for the brain-feature
// encoder (reference src/model/brain_feature_extractor.py:39-47, 56-68).
//
// The input projection gi = x W_ih^T + b_ih is a GEMM done beforehand (b2p_gemm); what is left
// is the latency-bound time recurrence. One launch per time step (both directions in one grid),
// driven by a host loop inside this library: a launch boundary is the cheapest correct grid-wide
// barrier at this size. Each block owns HU=8 hidden units x BB=8 batch rows of one direction,
// stages the 3*HU rows of W_hh and the BB rows of h_{t-1} in LDS and splits the K=H reduction
// over its four waves; wave 0 then applies the gate nonlinearities (fp32 throughout).
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {
constexpr int HU = 8;      // hidden units per block
constexpr int BB = 8;      // batch rows per block
constexpr int NTH = 256;   // 4 waves: K split in 4

// time index of processing step s for direction d
__device__ __forceinline__ int t_of(int s, int d, int T) { return d == 0 ? s : T - 1 - s; }

// ------------------------------------------------------------------ forward step
// gi [B][T][ndir*3H], whh [ndir][3H][H], bhh [ndir][3H], out [B][T][ndir*H],
// saved [B][T][ndir][4][H] (r, z, n, ghn)
__global__ void __launch_bounds__(NTH) gru_fwd_step(const float* __restrict__ gi, const float* __restrict__ whh,
                                                    const float* __restrict__ bhh, const float* __restrict__ h0,
                                                    float* __restrict__ out, float* __restrict__ saved, int B,
                                                    int T, int H, int ndir, int s) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int HP = H + 4;                       // padded row (float4 aligned, bank spread)
  float* Ws = sm;                             // [3*HU][HP]
  float* Hs = sm + 3 * HU * HP;               // [BB][HP]
  float* red = Hs + BB * HP;                  // [4][3][64]
  const int d = blockIdx.z;
  const int j0 = blockIdx.x * HU, b0 = blockIdx.y * BB;
  const int t = t_of(s, d, T);
  const int tprev = d == 0 ? t - 1 : t + 1;
  const int tid = threadIdx.x;
  const int H4 = H >> 2;
  const int G3 = 3 * H;

  // stage W rows (g*H + j0 + u) and h_{t-1} rows; the loads of a batch of SU float4 per thread are
  // issued back to back before their LDS stores (one memory latency per batch, not per element)
  const float* wd = whh + (int64_t)d * G3 * H;
  constexpr int SU = 8;
  const int nW = 3 * HU * H4, nH = BB * H4;
  for (int i0 = tid; i0 < nW + nH; i0 += NTH * SU) {
    float4 v[SU];
#pragma unroll
    for (int q = 0; q < SU; ++q) {
      const int i = i0 + q * NTH;
      v[q] = make_float4(0, 0, 0, 0);
      if (i < nW) {
        const int r = i / H4, c = i - r * H4;
        const int g = r / HU, u = r - g * HU;
        v[q] = reinterpret_cast<const float4*>(wd + (int64_t)(g * H + j0 + u) * H)[c];
      } else if (i < nW + nH) {
        const int r = (i - nW) / H4, c = (i - nW) - r * H4;
        const int b = b0 + r;
        if (b < B) {
          if (s == 0) {
            if (h0) v[q] = reinterpret_cast<const float4*>(h0 + ((int64_t)d * B + b) * H)[c];
          } else {
            v[q] = reinterpret_cast<const float4*>(out + ((int64_t)b * T + tprev) * ndir * H + (int64_t)d * H)[c];
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < SU; ++q) {
      const int i = i0 + q * NTH;
      if (i < nW) {
        const int r = i / H4, c = i - r * H4;
        reinterpret_cast<float4*>(Ws + r * HP)[c] = v[q];
      } else if (i < nW + nH) {
        const int r = (i - nW) / H4, c = (i - nW) - r * H4;
        reinterpret_cast<float4*>(Hs + r * HP)[c] = v[q];
      }
    }
  }
  __syncthreads();

  const int p = tid & 63, ks = tid >> 6;
  const int bl = p >> 3, u = p & 7;
  const int kq = H4 / 4;                    // float4 per quarter
  const float4* hr = reinterpret_cast<const float4*>(Hs + bl * HP) + ks * kq;
  const float4* wr = reinterpret_cast<const float4*>(Ws + (0 * HU + u) * HP) + ks * kq;
  const float4* wz = reinterpret_cast<const float4*>(Ws + (1 * HU + u) * HP) + ks * kq;
  const float4* wn = reinterpret_cast<const float4*>(Ws + (2 * HU + u) * HP) + ks * kq;
  float ar = 0.f, az = 0.f, an = 0.f;
  for (int c = 0; c < kq; ++c) {
    const float4 h = hr[c], a = wr[c], bz = wz[c], cn = wn[c];
    ar += h.x * a.x + h.y * a.y + h.z * a.z + h.w * a.w;
    az += h.x * bz.x + h.y * bz.y + h.z * bz.z + h.w * bz.w;
    an += h.x * cn.x + h.y * cn.y + h.z * cn.z + h.w * cn.w;
  }
  red[(ks * 3 + 0) * 64 + p] = ar;
  red[(ks * 3 + 1) * 64 + p] = az;
  red[(ks * 3 + 2) * 64 + p] = an;
  __syncthreads();
  if (ks != 0) return;
  const int b = b0 + bl, j = j0 + u;
  if (b >= B || j >= H) return;
  float gr = 0.f, gz = 0.f, gn = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    gr += red[(q * 3 + 0) * 64 + p];
    gz += red[(q * 3 + 1) * 64 + p];
    gn += red[(q * 3 + 2) * 64 + p];
  }
  const float* bd = bhh ? bhh + (int64_t)d * G3 : nullptr;
  if (bd) { gr += bd[j]; gz += bd[H + j]; gn += bd[2 * H + j]; }
  const float* gir = gi + ((int64_t)b * T + t) * ndir * G3 + (int64_t)d * G3;
  const float r = b2p_sigmoid(gir[j] + gr);
  const float z = b2p_sigmoid(gir[H + j] + gz);
  const float n = tanhf(gir[2 * H + j] + r * gn);
  const float hp = Hs[bl * HP + j];  // h_{t-1}[b][j]
  const float h = (1.f - z) * n + z * hp;
  out[((int64_t)b * T + t) * ndir * H + (int64_t)d * H + j] = h;
  float* sv = saved + (((int64_t)b * T + t) * ndir + d) * 4 * H;
  sv[j] = r;
  sv[H + j] = z;
  sv[2 * H + j] = n;
  sv[3 * H + j] = gn;
}

// ------------------------------------------------------------------ backward step
// Computes, for processing step s (going backwards), dh_s = dOut[t(s)] + [s < T-1] *
// (z_{s+1} * dh_{s+1} + W^T dgh_{s+1}) and from it the gate gradients at step s.
// dhbuf [ndir][B][H] holds dh of the step just processed (owner-local), dgh [B][T][ndir*3H].
__global__ void __launch_bounds__(NTH) gru_bwd_step(const float* __restrict__ dout, const float* __restrict__ whh,
                                                    const float* __restrict__ out, const float* __restrict__ saved,
                                                    const float* __restrict__ h0, float* __restrict__ dgi,
                                                    float* __restrict__ dgh, float* __restrict__ dhbuf,
                                                    float* __restrict__ dh0, int B, int T, int H, int ndir, int s,
                                                    int final_h0) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int G3 = 3 * H;
  const int GP = G3 + 4;
  float* Wt = sm;                 // [HU][GP]  column slice of W: Wt[u][g] = W[g][j0+u]
  float* Ds = sm + HU * GP;       // [BB][GP]  dgh_{s+1} rows
  float* red = Ds + BB * GP;      // [4][64]
  const int d = blockIdx.z;
  const int j0 = blockIdx.x * HU, b0 = blockIdx.y * BB;
  const int tid = threadIdx.x;
  const int p = tid & 63, ks = tid >> 6;
  const int bl = p >> 3, u = p & 7;
  const int b = b0 + bl, j = j0 + u;
  const bool has_next = final_h0 ? true : (s < T - 1);
  const int snext = final_h0 ? 0 : s + 1;       // step whose dgh feeds dh_s

  float rec = 0.f;
  if (has_next) {
    const int tn = t_of(snext, d, T);
    const float* wd = whh + (int64_t)d * G3 * H;
    // W column slice: per W row g, two float4 (units j0 .. j0+7) scattered into Wt[u][g]; dgh rows
    // as float4. Loads batched SU per thread ahead of their LDS stores (latency once per batch).
    constexpr int SU = 8;
    const int G34 = G3 >> 2;
    const int nW = 2 * G3, nD = BB * G34;
    for (int i0 = tid; i0 < nW + nD; i0 += NTH * SU) {
      float4 v[SU];
#pragma unroll
      for (int q = 0; q < SU; ++q) {
        const int i = i0 + q * NTH;
        v[q] = make_float4(0, 0, 0, 0);
        if (i < nW) {
          const int g = i >> 1, hf = i & 1;
          v[q] = *reinterpret_cast<const float4*>(wd + (int64_t)g * H + j0 + 4 * hf);
        } else if (i < nW + nD) {
          const int r = (i - nW) / G34, c = (i - nW) - r * G34;
          const int bb = b0 + r;
          if (bb < B) v[q] = reinterpret_cast<const float4*>(dgh + ((int64_t)bb * T + tn) * ndir * G3 + (int64_t)d * G3)[c];
        }
      }
#pragma unroll
      for (int q = 0; q < SU; ++q) {
        const int i = i0 + q * NTH;
        if (i < nW) {
          const int g = i >> 1, hf = i & 1;
          Wt[(4 * hf + 0) * GP + g] = v[q].x;
          Wt[(4 * hf + 1) * GP + g] = v[q].y;
          Wt[(4 * hf + 2) * GP + g] = v[q].z;
          Wt[(4 * hf + 3) * GP + g] = v[q].w;
        } else if (i < nW + nD) {
          const int r = (i - nW) / G34, c = (i - nW) - r * G34;
          reinterpret_cast<float4*>(Ds + r * GP)[c] = v[q];
        }
      }
    }
    __syncthreads();
    const int gq4 = G3 / 16;   // float4 per quarter of the reduction
    const float4* wr = reinterpret_cast<const float4*>(Wt + u * GP) + ks * gq4;
    const float4* dr = reinterpret_cast<const float4*>(Ds + bl * GP) + ks * gq4;
    float acc = 0.f;
    for (int g = 0; g < gq4; ++g) {
      const float4 a = wr[g], e = dr[g];
      acc += a.x * e.x + a.y * e.y + a.z * e.z + a.w * e.w;
    }
    red[ks * 64 + p] = acc;
    __syncthreads();
    if (ks != 0) return;
    rec = red[p] + red[64 + p] + red[128 + p] + red[192 + p];
  } else if (ks != 0) {
    return;
  }
  if (b >= B || j >= H) return;
  float* dhp = dhbuf + ((int64_t)d * B + b) * H + j;
  float dh;
  if (has_next) {
    const int tn = t_of(snext, d, T);
    const float zn = saved[(((int64_t)b * T + tn) * ndir + d) * 4 * H + H + j];
    dh = rec + zn * (*dhp);
  } else {
    dh = 0.f;
  }
  if (final_h0) {
    dh0[((int64_t)d * B + b) * H + j] = dh;
    return;
  }
  const int t = t_of(s, d, T);
  dh += dout[((int64_t)b * T + t) * ndir * H + (int64_t)d * H + j];
  *dhp = dh;
  const float* sv = saved + (((int64_t)b * T + t) * ndir + d) * 4 * H;
  const float r = sv[j], z = sv[H + j], n = sv[2 * H + j], ghn = sv[3 * H + j];
  float hprev;
  if (s == 0) hprev = h0 ? h0[((int64_t)d * B + b) * H + j] : 0.f;
  else hprev = out[((int64_t)b * T + (d == 0 ? t - 1 : t + 1)) * ndir * H + (int64_t)d * H + j];
  const float dn = dh * (1.f - z);
  const float dz = dh * (hprev - n);
  const float dan = dn * (1.f - n * n);
  const float dr = dan * ghn;
  const float dar = dr * r * (1.f - r);
  const float daz = dz * z * (1.f - z);
  float* gi_o = dgi + ((int64_t)b * T + t) * ndir * G3 + (int64_t)d * G3;
  float* gh_o = dgh + ((int64_t)b * T + t) * ndir * G3 + (int64_t)d * G3;
  gi_o[j] = dar; gi_o[H + j] = daz; gi_o[2 * H + j] = dan;
  gh_o[j] = dar; gh_o[H + j] = daz; gh_o[2 * H + j] = dan * r;
}

__global__ void gru_hprev_k(const float* __restrict__ out, const float* __restrict__ h0, float* __restrict__ hp,
                            int B, int T, int H, int ndir) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)ndir * B * T * H;
  if (i >= n) return;
  const int j = (int)(i % H);
  const int t = (int)((i / H) % T);
  const int b = (int)((i / ((int64_t)H * T)) % B);
  const int d = (int)(i / ((int64_t)H * T * B));
  const int tp = d == 0 ? t - 1 : t + 1;
  float v;
  if (tp < 0 || tp >= T) v = h0 ? h0[((int64_t)d * B + b) * H + j] : 0.f;
  else v = out[((int64_t)b * T + tp) * ndir * H + (int64_t)d * H + j];
  hp[i] = v;
}
}  // namespace

extern "C" int b2p_gru_fwd(const float* gi, const float* whh, const float* bhh, const float* h0, float* out,
                           float* saved, int64_t B, int64_t T, int64_t H, int ndir, b2p_stream_t stream) {
  B2P_CHECK_ARG(gi && whh && out && saved, "gru_fwd: NULL pointer");
  B2P_CHECK_ARG(H % (4 * 4) == 0 && H % HU == 0, "gru_fwd: hidden size must be a multiple of 16");
  B2P_CHECK_ARG(ndir == 1 || ndir == 2, "gru_fwd: ndir must be 1 or 2");
  if (B <= 0 || T <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int HP = (int)H + 4;
  const size_t shm = (size_t)(3 * HU * HP + BB * HP + 4 * 3 * 64) * sizeof(float);
  B2P_CHECK_ARG(shm <= 160 * 1024, "gru_fwd: hidden size too large for LDS staging");
  dim3 grid((unsigned)(H / HU), (unsigned)((B + BB - 1) / BB), (unsigned)ndir);
  for (int s = 0; s < (int)T; ++s) {
    hipLaunchKernelGGL(gru_fwd_step, grid, dim3(NTH), shm, st, gi, whh, bhh, h0, out, saved, (int)B, (int)T,
                       (int)H, ndir, s);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_gru_bwd(const float* dout, const float* whh, const float* out, const float* saved,
                           const float* h0, float* dgi, float* dgh, float* dh0, float* dhbuf, int64_t B,
                           int64_t T, int64_t H, int ndir, b2p_stream_t stream) {
  B2P_CHECK_ARG(dout && whh && out && saved && dgi && dgh && dhbuf, "gru_bwd: NULL pointer");
  B2P_CHECK_ARG(H % 16 == 0, "gru_bwd: hidden size must be a multiple of 16");
  B2P_CHECK_ARG(HU == 8, "gru_bwd: the W slice staging assumes 8 hidden units per block");
  B2P_CHECK_ARG(ndir == 1 || ndir == 2, "gru_bwd: ndir must be 1 or 2");
  if (B <= 0 || T <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int GP = 3 * (int)H + 4;
  const size_t shm = (size_t)(HU * GP + BB * GP + 4 * 64) * sizeof(float);
  B2P_CHECK_ARG(shm <= 160 * 1024, "gru_bwd: hidden size too large for LDS staging");
  dim3 grid((unsigned)(H / HU), (unsigned)((B + BB - 1) / BB), (unsigned)ndir);
  for (int s = (int)T - 1; s >= 0; --s) {
    hipLaunchKernelGGL(gru_bwd_step, grid, dim3(NTH), shm, st, dout, whh, out, saved, h0, dgi, dgh, dhbuf, dh0,
                       (int)B, (int)T, (int)H, ndir, s, 0);
  }
  if (dh0) {
    hipLaunchKernelGGL(gru_bwd_step, grid, dim3(NTH), shm, st, dout, whh, out, saved, h0, dgi, dgh, dhbuf, dh0,
                       (int)B, (int)T, (int)H, ndir, -1, 1);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_gru_hprev(const float* out, const float* h0, float* hp, int64_t B, int64_t T, int64_t H,
                             int ndir, b2p_stream_t stream) {
  B2P_CHECK_ARG(out && hp, "gru_hprev: NULL pointer");
  const int64_t n = (int64_t)ndir * B * T * H;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gru_hprev_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out, h0,
                     hp, (int)B, (int)T, (int)H, ndir);
  B2P_CHECK_LAUNCH();
  return 0;
}
