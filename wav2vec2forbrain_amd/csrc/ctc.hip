// Fused log_softmax + CTC loss (blank, reduction="mean", zero_infinity=True) and its gradient
// with respect to the logits, for src/model/w2v_custom_feat_extractor.py:59, 81-90 (torch
// nn.CTCLoss semantics: log-space alpha/beta over the 2S+1 extended label sequence; the loss of a
// sample is divided by its (clamped >= 1) target length and averaged over the batch; infeasible
// samples give loss 0 and gradient 0; frames t >= input_length get gradient 0).
//
// One workgroup per sample: the time recursion is sequential (barrier per frame) and the
// alpha/beta rows live in LDS while full alpha/beta tables go to the workspace for the
// per-(t, class) gradient pass.
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {
constexpr int NTH = 256;

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + logf(__expf(a - m) + __expf(b - m));
}
__device__ __forceinline__ float lse3(float a, float b, float c) {
  const float m = fmaxf(a, fmaxf(b, c));
  if (m == -INFINITY) return -INFINITY;
  return m + logf(__expf(a - m) + __expf(b - m) + __expf(c - m));
}

__global__ void __launch_bounds__(NTH) ctc_kernel(const float* __restrict__ logits, const int64_t* __restrict__ targets,
                                                  const int32_t* __restrict__ in_lens, const int64_t* __restrict__ tgt_lens,
                                                  int B, int T, int S, int C, int blank, float* __restrict__ nll_out,
                                                  float* __restrict__ grad, float* __restrict__ ws) {
  extern __shared__ float sm[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int Sp = 2 * S + 1;                         // max extended length
  float* lp = ws + (int64_t)b * ((int64_t)T * C + 2ll * T * Sp);
  float* alpha = lp + (int64_t)T * C;
  float* beta = alpha + (int64_t)T * Sp;
  int* lab = reinterpret_cast<int*>(sm);            // [Sp] extended labels
  float* rowA = sm + Sp;                            // [Sp]
  float* rowB = rowA + Sp;                          // [Sp]
  __shared__ float s_nll;

  int tl = (int)tgt_lens[b];
  if (tl < 0) tl = 0;
  if (tl > S) tl = S;
  int il = in_lens[b];
  if (il > T) il = T;
  if (il < 0) il = 0;
  const int L = 2 * tl + 1;
  const float* lg = logits + (int64_t)b * T * C;
  float* gr = grad + (int64_t)b * T * C;

  // log_softmax rows
  for (int t = tid; t < T; t += NTH) {
    const float* x = lg + (int64_t)t * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, x[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(x[c] - m);
    const float ls = m + logf(s);
    for (int c = 0; c < C; ++c) lp[(int64_t)t * C + c] = x[c] - ls;
  }
  for (int s = tid; s < L; s += NTH) {
    int l = (s & 1) ? (int)targets[(int64_t)b * S + (s >> 1)] : blank;
    lab[s] = (l < 0 || l >= C) ? blank : l;   // out-of-range ids cannot index log_probs
  }
  __syncthreads();

  float nll = INFINITY;
  if (il > 0) {
    // ---- alpha
    for (int s = tid; s < L; s += NTH) {
      float v = -INFINITY;
      if (s == 0) v = lp[blank];
      else if (s == 1) v = lp[lab[1]];
      rowA[s] = v;
      alpha[s] = v;
    }
    __syncthreads();
    float* prev = rowA;
    float* cur = rowB;
    for (int t = 1; t < il; ++t) {
      const float* lpt = lp + (int64_t)t * C;
      for (int s = tid; s < L; s += NTH) {
        const int l = lab[s];
        const float a1 = prev[s];
        const float a2 = s > 0 ? prev[s - 1] : -INFINITY;
        const float a3 = (s > 1 && l != blank && l != lab[s - 2]) ? prev[s - 2] : -INFINITY;
        const float v = lse3(a1, a2, a3);
        const float o = v == -INFINITY ? -INFINITY : v + lpt[l];
        cur[s] = o;
        alpha[(int64_t)t * Sp + s] = o;
      }
      __syncthreads();
      float* tmp = prev; prev = cur; cur = tmp;
    }
    if (tid == 0) {
      const float a = prev[L - 1];
      const float c = L > 1 ? prev[L - 2] : -INFINITY;
      s_nll = -lse2(a, c);
    }
    __syncthreads();   // the final alpha row is read above before rowA is reused for beta
    // ---- beta
    const float* lpl = lp + (int64_t)(il - 1) * C;
    for (int s = tid; s < L; s += NTH) {
      float v = -INFINITY;
      if (s == L - 1) v = lpl[blank];
      else if (s == L - 2) v = lpl[lab[s]];
      rowA[s] = v;   // prev (rowA) is free again after the barrier below
      beta[(int64_t)(il - 1) * Sp + s] = v;
    }
    __syncthreads();
    // note: `prev` may alias rowA; restart the ping-pong from rowA explicitly
    prev = rowA;
    cur = rowB;
    for (int t = il - 2; t >= 0; --t) {
      const float* lpt = lp + (int64_t)t * C;
      for (int s = tid; s < L; s += NTH) {
        const int l = lab[s];
        const float b1 = prev[s];
        const float b2 = s < L - 1 ? prev[s + 1] : -INFINITY;
        const float b3 = (s < L - 2 && l != blank && lab[s + 2] != l) ? prev[s + 2] : -INFINITY;
        const float v = lse3(b1, b2, b3);
        const float o = v == -INFINITY ? -INFINITY : v + lpt[l];
        cur[s] = o;
        beta[(int64_t)t * Sp + s] = o;
      }
      __syncthreads();
      float* tmp = prev; prev = cur; cur = tmp;
    }
    __syncthreads();
    nll = s_nll;
  }
  if (tid == 0) nll_out[b] = nll;

  // ---- gradient wrt logits of loss_b * gscale, gscale = 1 / (B * max(tl,1))
  const bool inf = !(nll < INFINITY);
  const float gscale = 1.0f / ((float)B * (float)(tl > 1 ? tl : 1));
  for (int i = tid; i < T * C; i += NTH) {
    const int t = i / C, c = i - t * C;
    gr[i] = 0.f;
    (void)c;
  }
  __syncthreads();
  if (inf || il == 0) return;
  // g_lp[t][c] = exp(lp) - exp(lcab + nll - lp); then grad = g - softmax * sum_c g
  for (int t = tid; t < il; t += NTH) {
    const float* lpt = lp + (int64_t)t * C;
    const float* at = alpha + (int64_t)t * Sp;
    const float* bt = beta + (int64_t)t * Sp;
    float* gt = gr + (int64_t)t * C;
    float gsum = 0.f;
    for (int c = 0; c < C; ++c) {
      // online logsumexp over states with label c
      float m = -INFINITY, acc = 0.f;
      for (int s = (c == blank ? 0 : 1); s < L; s += (c == blank ? 2 : 1)) {
        if (lab[s] != c) continue;
        const float v = at[s] + bt[s];
        if (v == -INFINITY) continue;
        if (v > m) { acc = acc * __expf(m - v) + 1.f; m = v; }
        else acc += __expf(v - m);
      }
      const float lcab = m == -INFINITY ? -INFINITY : m + logf(acc);
      const float e = __expf(lpt[c]);
      const float g = (e - (lcab == -INFINITY ? 0.f : __expf(lcab + nll - lpt[c]))) * gscale;
      gt[c] = g;
      gsum += g;
    }
    for (int c = 0; c < C; ++c) gt[c] = gt[c] - __expf(lpt[c]) * gsum;
  }
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
  const int64_t Sp = 2 * S + 1;
  const size_t shm = (size_t)3 * Sp * sizeof(float);
  B2P_CHECK_ARG(shm <= 64 * 1024, "ctc: target length too large");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ctc_kernel, dim3((unsigned)B), dim3(NTH), shm, st, logits, targets, in_lens, tgt_lens, (int)B,
                     (int)T, (int)S, (int)C, blank, nll, grad_logits, workspace);
  hipLaunchKernelGGL(ctc_loss_mean, dim3(1), dim3(64), 0, st, nll, tgt_lens, (int)B, (int)S, loss);
  B2P_CHECK_LAUNCH();
  return 0;
}
