// On-device CTC prefix beam search without a language model (config 5's "on-device CTC
// beam decode"). The reference decodes test predictions on the host with pyctcdecode through
// Wav2Vec2ProcessorWithLM (src/train/evaluator.py:148-154,189-210; beam_width / beam_prune_logp /
// token_min_logp from src/experiments/b2t_gru_w2v_experiment.py:66-71); its KenLM / processor
// assets are unavailable offline, so this is the LM-free prefix beam search (Hannun et al. 2014)
// with pyctcdecode's two pruning rules, restated exactly by oracle/ctc_beam_oracle.py.
//
// Per frame t, every live beam (prefix l, log p_b, log p_nb) proposes C candidates k = w*C + c:
//   c == blank : l stays,      b = lse(p_b, p_nb) + y_blank,   nb = p_nb + y_last (-inf if l empty)
//   c == last  : l + c,        nb = p_b + y_c
//   otherwise  : l + c,        nb = lse(p_b, p_nb) + y_c
// An extension that equals another live beam's prefix (l' = l + c) is merged into that beam's stay
// candidate (nb log-added) and suppressed. Characters with y_c < token_min_logp are skipped unless c
// is the frame's argmax; candidates below best + beam_prune_logp are dropped; the W best (ties: lower
// k) become the next beams. Prefixes are identified by a 64-bit hash chain; a (parent, char) record
// per frame and beam lets the best beam's tokens be read back at the end.
//
// One 256-thread workgroup per sample; W <= 128, C <= 64; log-softmax of the logits row in-kernel.
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {

constexpr int BM_W = 128;
constexpr int BM_C = 64;
constexpr int BM_N = BM_W * BM_C;   // candidate slots (sorted bitonically)
constexpr float NEG = -INFINITY;

__device__ __forceinline__ float lse2(float a, float b) {
  if (a == NEG) return b;
  if (b == NEG) return a;
  const float m = fmaxf(a, b);
  return m + log1pf(expf(-fabsf(a - b)));
}
__device__ __forceinline__ uint64_t hmix(uint64_t h, int c) { return (h ^ (uint64_t)(c + 1)) * 0x100000001B3ull; }
// float -> uint32 with the same order (for the descending-score sort key)
__device__ __forceinline__ uint32_t ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(256) ctc_beam_k(const float* __restrict__ logits, int T, int C,
                                                  const int32_t* __restrict__ lens, int W, int blank,
                                                  float token_min_logp, float prune_logp,
                                                  int32_t* __restrict__ hist, int32_t* __restrict__ out_tok,
                                                  int32_t* __restrict__ out_len, float* __restrict__ out_score) {
  __shared__ float y[BM_C];
  __shared__ float pb[BM_W], pnb[BM_W];
  __shared__ uint64_t hs[BM_W], phs[BM_W];
  __shared__ int last[BM_W], blen[BM_W];
  __shared__ float cb[BM_N], cnb[BM_N];
  __shared__ uint64_t key[BM_N];
  __shared__ float sh_red[256];
  __shared__ int sh_arg;
  __shared__ float sh_best;
  // next-beam staging
  __shared__ float npb[BM_W], npnb[BM_W];
  __shared__ uint64_t nhs[BM_W], nphs[BM_W];
  __shared__ int nlast[BM_W], nlen[BM_W];

  const int b = blockIdx.x, tid = threadIdx.x;
  const int Tb = lens ? min(max(lens[b], 0), T) : T;
  const float* lg = logits + (int64_t)b * T * C;
  int32_t* hb = hist + (int64_t)b * T * W;
  const int N = W * C;
  int np2 = 1;
  while (np2 < N) np2 <<= 1;

  for (int w = tid; w < W; w += 256) {
    pb[w] = w == 0 ? 0.f : NEG;
    pnb[w] = NEG;
    hs[w] = 0xCBF29CE484222325ull;
    phs[w] = 0;
    last[w] = -1;
    blen[w] = 0;
  }
  __syncthreads();
  for (int t = 0; t < Tb; ++t) {
    // log-softmax of frame t (C <= 64: one wave) and its argmax
    if (tid < 64) {
      const float v = tid < C ? lg[(int64_t)t * C + tid] : NEG;
      float m = v;
      int am = tid < C ? tid : 1 << 30;
      for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64);
        const int a2 = __shfl_xor(am, o, 64);
        if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
      }
      float s = tid < C ? expf(v - m) : 0.f;
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (tid < C) y[tid] = v - m - logf(s);
      if (tid == 0) sh_arg = am;
    }
    __syncthreads();
    const int arg = sh_arg;
    // candidates
    for (int k = tid; k < np2; k += 256) {
      float vb = NEG, vnb = NEG;
      if (k < N) {
        const int w = k / C, c = k - w * C;
        const float tot = lse2(pb[w], pnb[w]);
        const bool use = y[c] >= token_min_logp || c == arg;
        if (tot != NEG) {
          if (c == blank) {   // the stay candidate: blank path (if blank is used) + repeat path (if last is)
            if (use) vb = tot + y[blank];
            const int l = last[w];
            if (l >= 0 && (y[l] >= token_min_logp || l == arg)) vnb = pnb[w] + y[l];
          } else if (use) {
            vnb = (c == last[w] ? pb[w] : tot) + y[c];
          }
        }
      }
      cb[k] = vb;
      cnb[k] = vnb;
    }
    __syncthreads();
    // merge: beam w (prefix l' = l + last) absorbs the extension (w0, last) of its parent beam w0
    for (int w = tid; w < W; w += 256) {
      const int l = last[w];
      if (blen[w] == 0 || lse2(pb[w], pnb[w]) == NEG || !(y[l] >= token_min_logp || l == arg)) continue;
      for (int w0 = 0; w0 < W; ++w0) {
        if (w0 != w && hs[w0] == phs[w] && lse2(pb[w0], pnb[w0]) != NEG) {
          const int ke = w0 * C + l;
          cnb[w * C + blank] = lse2(cnb[w * C + blank], cnb[ke]);
          break;
        }
      }
    }
    __syncthreads();
    for (int w = tid; w < W; w += 256) {   // suppress the merged extensions (after every merge read them)
      const int l = last[w];
      if (blen[w] == 0 || lse2(pb[w], pnb[w]) == NEG || !(y[l] >= token_min_logp || l == arg)) continue;
      for (int w0 = 0; w0 < W; ++w0)
        if (w0 != w && hs[w0] == phs[w] && lse2(pb[w0], pnb[w0]) != NEG) {
          cb[w0 * C + l] = NEG;
          cnb[w0 * C + l] = NEG;
          break;
        }
    }
    __syncthreads();
    // best total, prune threshold
    float mx = NEG;
    for (int k = tid; k < N; k += 256) mx = fmaxf(mx, lse2(cb[k], cnb[k]));
    sh_red[tid] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) sh_red[tid] = fmaxf(sh_red[tid], sh_red[tid + s]);
      __syncthreads();
    }
    if (tid == 0) sh_best = sh_red[0];
    __syncthreads();
    const float thr = sh_best + prune_logp;
    for (int k = tid; k < np2; k += 256) {
      const float tot = k < N ? lse2(cb[k], cnb[k]) : NEG;
      const bool ok = tot != NEG && tot >= thr;
      // ascending sort of (descending score, ascending k); dropped candidates last
      key[k] = ok ? ((uint64_t)(~ord(tot)) << 32) | (uint32_t)k : ~0ull;
    }
    __syncthreads();
    for (int size = 2; size <= np2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < np2 / 2; i += 256) {
          const int lo = 2 * i - (i & (stride - 1));
          const int hi = lo + stride;
          const bool asc = (lo & size) == 0;
          const uint64_t a = key[lo], c2 = key[hi];
          if ((a > c2) == asc) {
            key[lo] = c2;
            key[hi] = a;
          }
        }
        __syncthreads();
      }
    }
    // next beams
    for (int w = tid; w < W; w += 256) {
      const uint64_t kk = key[w];
      int32_t rec = -1;
      if (kk == ~0ull) {
        npb[w] = NEG;
        npnb[w] = NEG;
        nhs[w] = 0;
        nphs[w] = 0;
        nlast[w] = -1;
        nlen[w] = 0;
      } else {
        const int k = (int)(uint32_t)kk;
        const int w0 = k / C, c = k - w0 * C;
        npb[w] = cb[k];
        npnb[w] = cnb[k];
        if (c == blank) {
          nhs[w] = hs[w0];
          nphs[w] = phs[w0];
          nlast[w] = last[w0];
          nlen[w] = blen[w0];
          rec = w0 << 8 | 0xFF;
        } else {
          nhs[w] = hmix(hs[w0], c);
          nphs[w] = hs[w0];
          nlast[w] = c;
          nlen[w] = blen[w0] + 1;
          rec = w0 << 8 | c;
        }
      }
      hb[(int64_t)t * W + w] = rec;
    }
    __syncthreads();
    for (int w = tid; w < W; w += 256) {
      pb[w] = npb[w];
      pnb[w] = npnb[w];
      hs[w] = nhs[w];
      phs[w] = nphs[w];
      last[w] = nlast[w];
      blen[w] = nlen[w];
    }
    __syncthreads();
  }
  // read back the best beam (beam 0 after the last sort; empty prefix when Tb == 0)
  __threadfence_block();
  if (tid == 0) {
    const int n = Tb > 0 ? blen[0] : 0;
    out_len[b] = n;
    out_score[b] = Tb > 0 ? lse2(pb[0], pnb[0]) : 0.f;
    int w = 0, pos = n;
    for (int t = Tb - 1; t >= 0 && pos > 0; --t) {
      const int32_t rec = hb[(int64_t)t * W + w];
      const int c = rec & 0xFF;
      if (c != 0xFF) out_tok[(int64_t)b * T + (--pos)] = c;
      w = rec >> 8;
    }
    for (int i = n; i < T; ++i) out_tok[(int64_t)b * T + i] = -1;
  }
}

}  // namespace

extern "C" int64_t b2p_ctc_beam_workspace(int64_t B, int64_t T, int64_t beam) { return B * T * beam; }

extern "C" int b2p_ctc_prefix_beam(const float* logits, int64_t B, int64_t T, int64_t C, const int32_t* lens,
                                   int64_t beam, int blank, float token_min_logp, float beam_prune_logp,
                                   int32_t* workspace, int32_t* out_tokens, int32_t* out_len, float* out_score,
                                   b2p_stream_t stream) {
  B2P_CHECK_ARG(logits && workspace && out_tokens && out_len && out_score, "ctc_prefix_beam: NULL pointer");
  B2P_CHECK_ARG(beam >= 1 && beam <= BM_W, "ctc_prefix_beam: beam width must be in [1, %d]", BM_W);
  B2P_CHECK_ARG(C >= 2 && C <= BM_C && blank >= 0 && blank < C, "ctc_prefix_beam: need 2 <= C <= %d, blank < C",
                BM_C);
  B2P_CHECK_ARG(T >= 0 && beam_prune_logp <= 0.f, "ctc_prefix_beam: T >= 0, beam_prune_logp <= 0");
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ctc_beam_k, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, logits, (int)T, (int)C, lens,
                     (int)beam, blank, token_min_logp, beam_prune_logp, workspace, out_tokens, out_len, out_score);
  B2P_CHECK_LAUNCH();
  return 0;
}
