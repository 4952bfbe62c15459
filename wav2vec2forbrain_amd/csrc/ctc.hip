// Fused log_softmax + CTC loss (blank, reduction="mean", zero_infinity=True) and its gradient
// with respect to the logits, for src/model/w2v_custom_feat_extractor.py:59, 81-90 (torch
// nn.CTCLoss semantics: log-space alpha/beta over the 2S+1 extended label sequence; the loss of a
// sample is divided by its (clamped >= 1) target length and averaged over the batch; infeasible
// samples give loss 0 and gradient 0; frames t >= input_length get gradient 0).
//
// Three launches, all latency-shaped for gfx950's 64-wide wavefronts:
//  1. ctc_lsm_k   log_softmax of every (b, t) row into the workspace (one wave per row group).
//  2. ctc_ab_k    grid (B, 2): ONE wavefront per sample and direction runs the whole alpha (or
//                 beta) recursion out of registers — lane l owns extended states 4l..4l+3 (NS per
//                 lane in general), the s-1 / s-2 neighbours of its first states come from lane l-1
//                 by two cross-lane shuffles, the sample's log-prob rows sit in LDS. No workgroup
//                 barrier per frame; alpha and beta run concurrently.
//  3. ctc_grad_k  one wave per (b, t): logsumexp of alpha+beta per class via LDS atomics, then
//                 grad = softmax - exp(lcab + nll - lp) scaled by 1 / (B * max(tl, 1)).
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {

__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m) + __expf(c - m));
}
__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + __logf(__expf(a - m) + __expf(b - m));
}

struct SampleInfo {
  int tl, il, L;
};
__device__ __forceinline__ SampleInfo sample_info(const int32_t* in_lens, const int64_t* tgt_lens, int b, int T,
                                                  int S) {
  SampleInfo si;
  int tl = (int)tgt_lens[b];
  si.tl = tl < 0 ? 0 : (tl > S ? S : tl);
  int il = in_lens[b];
  si.il = il < 0 ? 0 : (il > T ? T : il);
  si.L = 2 * si.tl + 1;
  return si;
}
// extended label of state s (blank at even s); ids outside [0, C) cannot index log_probs -> blank
__device__ __forceinline__ int ext_label(const int64_t* tg, int s, int blank, int C) {
  if (!(s & 1)) return blank;
  const int64_t l = tg[s >> 1];
  return (l < 0 || l >= C) ? blank : (int)l;
}

// ---------------------------------------------------------------------------- 1. log_softmax
// one thread per (b, t) row (C small: 32 classes)
__global__ void ctc_lsm_k(const float* __restrict__ logits, float* __restrict__ ws, int64_t rows, int T, int C,
                          int64_t per_sample) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const int64_t b = r / T, t = r - b * T;
  const float* x = logits + r * C;
  float m = -INFINITY;
  for (int c = 0; c < C; ++c) m = fmaxf(m, x[c]);
  float s = 0.f;
  for (int c = 0; c < C; ++c) s += __expf(x[c] - m);
  const float ls = m + __logf(s);
  float* lp = ws + b * per_sample + t * C;
  for (int c = 0; c < C; ++c) lp[c] = x[c] - ls;
}

// ---------------------------------------------------------------------------- 2. alpha / beta
template <int NS>
__global__ void __launch_bounds__(64) ctc_ab_k(const int64_t* __restrict__ targets, const int32_t* __restrict__ in_lens,
                                               const int64_t* __restrict__ tgt_lens, int T, int S, int C, int blank,
                                               float* __restrict__ ws, float* __restrict__ nll_out) {
  extern __shared__ float lps[];   // [T][C] log-probs of this sample
  const int b = blockIdx.x, dir = blockIdx.y, lane = threadIdx.x;
  const int Sp = 2 * S + 1;
  const int64_t per_sample = (int64_t)T * C + 2ll * T * Sp;
  float* lp = ws + (int64_t)b * per_sample;
  float* tab = lp + (int64_t)T * C + (dir ? (int64_t)T * Sp : 0);   // alpha (dir 0) or beta (dir 1)
  const SampleInfo si = sample_info(in_lens, tgt_lens, b, T, S);
  const int L = si.L, il = si.il;
  const int64_t* tg = targets + (int64_t)b * S;
  for (int i = lane; i < T * C; i += 64) lps[i] = lp[i];

  // per-state constants: label, skip-allowed (alpha: s-2 -> s; beta: s+2 -> s)
  int lab[NS];
  bool skip[NS], valid[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int s = NS * lane + j;
    valid[j] = s < L;
    lab[j] = valid[j] ? ext_label(tg, s, blank, C) : blank;
    if (dir == 0) skip[j] = valid[j] && s > 1 && lab[j] != blank && lab[j] != ext_label(tg, s - 2, blank, C);
    else skip[j] = valid[j] && s < L - 2 && lab[j] != blank && lab[j] != ext_label(tg, s + 2, blank, C);
  }
  __syncthreads();
  if (il == 0) {
    if (dir == 0 && lane == 0) nll_out[b] = INFINITY;
    return;
  }
  float v[NS];
  const int t0 = dir == 0 ? 0 : il - 1;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int s = NS * lane + j;
    float x = -INFINITY;
    if (dir == 0 && (s == 0 || s == 1) && s < L) x = lps[t0 * C + lab[j]];
    if (dir == 1 && (s == L - 1 || s == L - 2) && s >= 0) x = lps[t0 * C + lab[j]];
    v[j] = x;
    if (valid[j]) tab[(int64_t)t0 * Sp + s] = x;
  }
  for (int k = 1; k < il; ++k) {
    const int t = dir == 0 ? k : il - 1 - k;
    float nv[NS];
    if (dir == 0) {
      // neighbours s-1, s-2 of this lane's first states live in lane-1
      const float p1 = __shfl_up(v[NS - 1], 1, 64);
      float p2;
      if constexpr (NS >= 2) p2 = __shfl_up(v[NS - 2], 1, 64);
      else p2 = __shfl_up(v[0], 2, 64);
      const float q1 = lane > 0 ? p1 : -INFINITY;
      const float q2 = lane > (NS >= 2 ? 0 : 1) ? p2 : -INFINITY;
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const float a1 = v[j];
        const float a2 = j >= 1 ? v[j >= 1 ? j - 1 : 0] : q1;
        const float a3 = skip[j] ? (j >= 2 ? v[j >= 2 ? j - 2 : 0] : (j == 1 ? q1 : q2)) : -INFINITY;
        const float o = lse3(a1, a2, a3);
        nv[j] = (valid[j] && o != -INFINITY) ? o + lps[t * C + lab[j]] : -INFINITY;
      }
    } else {
      // neighbours s+1, s+2 of this lane's last states live in lane+1
      const float p1 = __shfl_down(v[0], 1, 64);
      float p2;
      if constexpr (NS >= 2) p2 = __shfl_down(v[1], 1, 64);
      else p2 = __shfl_down(v[0], 2, 64);
      const float q1 = lane < 63 ? p1 : -INFINITY;
      const float q2 = lane < (NS >= 2 ? 63 : 62) ? p2 : -INFINITY;
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const float b1 = v[j];
        const float b2 = j + 1 < NS ? v[j + 1 < NS ? j + 1 : 0] : q1;
        const float b3 = skip[j] ? (j + 2 < NS ? v[j + 2 < NS ? j + 2 : 0] : (j + 1 < NS ? q1 : q2)) : -INFINITY;
        const float o = lse3(b1, b2, b3);
        nv[j] = (valid[j] && o != -INFINITY) ? o + lps[t * C + lab[j]] : -INFINITY;
      }
    }
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      v[j] = nv[j];
      if (valid[j]) tab[(int64_t)t * Sp + NS * lane + j] = nv[j];
    }
  }
  if (dir == 0) {
    // nll = -logsumexp(alpha[il-1][L-1], alpha[il-1][L-2]): gather the two end states
    float e1 = -INFINITY, e2 = -INFINITY;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int s = NS * lane + j;
      if (s == L - 1) e1 = v[j];
      if (s == L - 2) e2 = v[j];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      e1 = fmaxf(e1, __shfl_xor(e1, o, 64));
      e2 = fmaxf(e2, __shfl_xor(e2, o, 64));
    }
    if (lane == 0) nll_out[b] = -lse2(e1, e2);
  }
}

// ---------------------------------------------------------------------------- 3. gradient
// grid (B, ceil(T/4)), 4 waves: wave w handles frame t = 4*blockIdx.y + w
template <int NS>
__global__ void __launch_bounds__(256) ctc_grad_k(const int64_t* __restrict__ targets, const int32_t* __restrict__ in_lens,
                                                  const int64_t* __restrict__ tgt_lens, int B, int T, int S, int C,
                                                  int blank, const float* __restrict__ ws,
                                                  const float* __restrict__ nll_in, float* __restrict__ grad) {
  __shared__ float acc[4][64];
  const int b = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = 4 * blockIdx.y + w;
  if (t >= T) return;
  const int Sp = 2 * S + 1;
  const int64_t per_sample = (int64_t)T * C + 2ll * T * Sp;
  const float* lp = ws + (int64_t)b * per_sample + (int64_t)t * C;
  const float* at = ws + (int64_t)b * per_sample + (int64_t)T * C + (int64_t)t * Sp;
  const float* bt = at + (int64_t)T * Sp;
  float* gt = grad + ((int64_t)b * T + t) * C;
  const SampleInfo si = sample_info(in_lens, tgt_lens, b, T, S);
  const float nll = nll_in[b];
  if (!(nll < INFINITY) || t >= si.il) {   // infeasible sample (zero_infinity) or t >= input length
    for (int c = lane; c < C; c += 64) gt[c] = 0.f;
    return;
  }
  const int64_t* tg = targets + (int64_t)b * S;
  float vs[NS];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int s = NS * lane + j;
    vs[j] = s < si.L ? at[s] + bt[s] : -INFINITY;
    m = fmaxf(m, vs[j]);
  }
  m = warp_max(m);
  for (int c = lane; c < 64; c += 64) acc[w][c] = 0.f;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int s = NS * lane + j;
    if (vs[j] != -INFINITY) atomicAdd(&acc[w][ext_label(tg, s, blank, C)], __expf(vs[j] - m));
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const float gscale = 1.0f / ((float)B * (float)(si.tl > 1 ? si.tl : 1));
  // classes c = lane (C <= 64, checked on the host)
  float g = 0.f, e = 0.f;
  if (lane < C) {
    const float l = lp[lane];
    const float a = acc[w][lane];
    const float lcab = (a > 0.f && m != -INFINITY) ? m + __logf(a) : -INFINITY;
    e = __expf(l);
    g = (e - (lcab == -INFINITY ? 0.f : __expf(lcab + nll - l))) * gscale;
  }
  const float gsum = warp_sum(g);
  if (lane < C) gt[lane] = g - e * gsum;
}

__global__ void ctc_loss_mean(const float* __restrict__ nll, const int64_t* __restrict__ tgt_lens, int B, int S,
                              float* __restrict__ loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) {
    const float v = nll[b];
    if (!(v < INFINITY)) continue;    // zero_infinity
    int tl = (int)tgt_lens[b];
    if (tl > S) tl = S;
    s += v / (float)(tl > 1 ? tl : 1);
  }
  *loss = s / (float)B;
}

template <int NS>
int launch_ab_grad(const int64_t* targets, const int32_t* in_lens, const int64_t* tgt_lens, int64_t B, int64_t T,
                   int64_t S, int64_t C, int blank, float* nll, float* grad, float* ws, hipStream_t st) {
  const size_t shm = (size_t)T * C * sizeof(float);
  static bool attr = false;
  if (!attr) {
    B2P_CHECK_HIP(hipFuncSetAttribute((const void*)ctc_ab_k<NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(ctc_ab_k<NS>, dim3((unsigned)B, 2), dim3(64), shm, st, targets, in_lens, tgt_lens, (int)T,
                     (int)S, (int)C, blank, ws, nll);
  hipLaunchKernelGGL(ctc_grad_k<NS>, dim3((unsigned)B, (unsigned)((T + 3) / 4)), dim3(256), 0, st, targets, in_lens,
                     tgt_lens, (int)B, (int)T, (int)S, (int)C, blank, ws, nll, grad);
  return 0;
}
}  // namespace

extern "C" int64_t b2p_ctc_workspace(int64_t B, int64_t T, int64_t S, int64_t C) {
  return B * (T * C + 2 * T * (2 * S + 1));
}

extern "C" int b2p_ctc_fwd_bwd(const float* logits, const int64_t* targets, const int32_t* in_lens,
                               const int64_t* tgt_lens, int64_t B, int64_t T, int64_t S, int64_t C, int blank,
                               float* nll, float* loss, float* grad_logits, float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(logits && targets && in_lens && tgt_lens && nll && loss && grad_logits && workspace,
                "ctc: NULL pointer");
  B2P_CHECK_ARG(blank >= 0 && blank < C, "ctc: blank out of range");
  B2P_CHECK_ARG(S >= 0 && T > 0 && C > 0 && B > 0, "ctc: bad sizes");
  B2P_CHECK_ARG(C <= 64, "ctc: at most 64 classes (vocabulary of the CTC head: 32)");
  B2P_CHECK_ARG(T * C * 4 <= 160 * 1024, "ctc: T * C log-probs of a sample must fit in LDS (160 KB)");
  B2P_CHECK_ARG(2 * S + 1 <= 64 * 8, "ctc: target length too large (2S+1 <= 512)");
  hipStream_t st = (hipStream_t)stream;
  const int64_t rows = B * T;
  const int64_t per_sample = T * C + 2 * T * (2 * S + 1);
  hipLaunchKernelGGL(ctc_lsm_k, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, logits, workspace, rows,
                     (int)T, (int)C, per_sample);
  const int64_t L = 2 * S + 1;
  int rc;
  if (L <= 64) rc = launch_ab_grad<1>(targets, in_lens, tgt_lens, B, T, S, C, blank, nll, grad_logits, workspace, st);
  else if (L <= 128) rc = launch_ab_grad<2>(targets, in_lens, tgt_lens, B, T, S, C, blank, nll, grad_logits, workspace, st);
  else if (L <= 256) rc = launch_ab_grad<4>(targets, in_lens, tgt_lens, B, T, S, C, blank, nll, grad_logits, workspace, st);
  else rc = launch_ab_grad<8>(targets, in_lens, tgt_lens, B, T, S, C, blank, nll, grad_logits, workspace, st);
  if (rc) return rc;
  hipLaunchKernelGGL(ctc_loss_mean, dim3(1), dim3(64), 0, st, nll, tgt_lens, (int)B, (int)S, loss);
  B2P_CHECK_LAUNCH();
  return 0;
}
