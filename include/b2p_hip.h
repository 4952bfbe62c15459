/*
 * b2p_hip.h — C ABI of the MI355X-native (gfx950 / CDNA4) b2p2t_gru+w2v training-step kernels.
 *
 * The reference (yuanhao-chen-nyoeghau/Wav2Vec2ForBrain) is pure Python on PyTorch/HF transformers:
 * it has no FFI. Its hot path is the per-batch body of Trainer._train_epoch
 * (src/train/train_loop.py:41-84) calling W2VBrainEncoderModel.forward
 * (src/model/w2v_custom_feat_extractor.py:65-122). Every entry point below replaces one
 * third-party operator that path reaches; the reference call site is cited per entry.
 * The "binding a maintainer would add" is the ctypes layer in
 * wav2vec2forbrain_amd/_lib.py.
 *
 * Conventions
 *  - raw device pointers (fp32 activations/weights/grads, int64 indices) + explicit sizes;
 *    the caller (PyTorch caching allocator) owns every buffer, workspaces included;
 *  - `stream` is a hipStream_t; all work is stream-ordered, no host synchronisation,
 *    no allocation on the hot path (graph-capturable);
 *  - return 0 on success, nonzero on error; b2p_last_error() returns the message
 *    (thread-local, valid until the next failing call on that thread).
 */
#ifndef B2P_HIP_H
#define B2P_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* b2p_stream_t; /* hipStream_t */

/* ------------------------------------------------------------------ library */
const char* b2p_last_error(void);
int b2p_version(void);
/* sizeof(b2p_operand), sizeof(b2p_epilogue), sizeof(b2p_gemm_desc): lets a binding verify its
 * struct layouts against the compiled library. */
int b2p_abi_sizes(int64_t* out3);
/* optional per-kernel-family HIP-event timing (bench.py roofline): family ids in
 * wav2vec2forbrain_amd/_lib.py. enable=0 turns it off. */
int b2p_timing_enable(int family, int max_events);
int b2p_timing_read(int family, float* total_ms, int* count, double* total_flops);

/* ------------------------------------------------------------------ GEMM
 * C[z](m,n) = epilogue( alpha * sum_k A[z](m,k) * B[z](k,n) ), bf16 MFMA (fp32 accumulate)
 * or exact-fp32 MFMA (precision=1). Operands are fp32 in HBM (converted while being staged
 * into LDS) or bf16 in HBM (copied straight into LDS by global_load_lds, transposed on the LDS
 * read with ds_read_b64_tr_b16 when the operand's contiguous dimension is m/n). Replaces every nn.Linear / matmul / conv-as-GEMM of the path:
 *   nn.Linear (TF w2v q/k/v/out_proj, FFN, lm_head: modeling_wav2vec2.py Wav2Vec2Attention,
 *   Wav2Vec2FeedForward; src/model/w2v_custom_feat_extractor.py:152;
 *   src/util/nn_helper.py:31-49 create_fully_connected),
 *   einsum("btd,bdk->btk") day layer (src/model/b2p2t_model.py:155-158, via gather1 = day_idxs),
 *   nn.Unfold + GRU input projection (src/model/b2p2t_model.py:162-167 +
 *   src/model/brain_feature_extractor.py:39-47, via the implicit conv view),
 *   grouped positional Conv1d (modeling_wav2vec2.py Wav2Vec2PositionalConvEmbedding, implicit
 *   conv view), attention QK^T / PV (eager_attention_forward).
 */
typedef struct {
  const void* ptr;       /* fp32 (dtype 0) or bf16 (dtype 1) elements                   */
  int64_t ld;            /* elements between consecutive outer indices                 */
  int64_t bs1, bs2;      /* batch strides for z1 = z / nz2 and z2 = z % nz2            */
  const int64_t* gather1;/* optional: offset uses gather1[z1] * bs1 instead of z1*bs1  */
  int32_t inner_is_k;    /* 1: the contiguous dimension is the reduction dimension     */
  int32_t conv;          /* 1: implicit conv1d view (below)                           */
  /* implicit conv1d view: logical element (r, j) with r = b*conv_T_out + t and
   * j = tap*conv_Cg + ch maps to src[b*conv_sample_stride + (t*conv_stride + tap - conv_pad)*ld + ch],
   * zero when the frame index falls outside [0, conv_T_in). */
  int32_t conv_T_out, conv_T_in, conv_stride, conv_pad, conv_Cg;
  int32_t dtype;         /* 0 = fp32 (converted while staged into LDS), 1 = bf16: both operands
                          * bf16 selects the LDS-DMA kernel (global_load_lds, ptr/ld/bs/Cg
                          * multiples of 8 elements, K % 8 == 0 for a k-contiguous operand);
                          * 2 = fp16 (precision 2 only): the same kernel on fp16 MFMA, plain
                          * (non-conv) operands                                               */
  int64_t conv_sample_stride;
} b2p_operand;

enum { B2P_ACT_NONE = 0, B2P_ACT_GELU = 1, B2P_ACT_SOFTSIGN = 2, B2P_ACT_SILU = 3 };
enum { B2P_EPI_C16_FP16 = 1 };

typedef struct {
  float* C;
  int64_t ldc, cbs1, cbs2;
  float alpha, beta;          /* beta != 0: C = alpha*acc + beta*C_old                        */
  const float* bias;          /* [N] added after alpha/beta, or NULL                          */
  int64_t biasbs1;            /* bias offset per z1 (grouped GEMMs)                           */
  const int64_t* bias_gather; /* optional: bias offset = bias_gather[z1] * biasbs1 (day bias)  */
  float* pre_out;             /* optional: store the pre-activation value (layout of C)       */
  int32_t act;                /* B2P_ACT_* applied after bias                                  */
  int32_t act_bwd;            /* B2P_ACT_*: multiply by act'(aux) after dropout (backward)     */
  const float* aux;           /* pre-activation for act_bwd                                    */
  int64_t ldaux, abs1, abs2;
  float drop_p;               /* dropout probability (0 = off); mask = f(drop_seed, index)     */
  int32_t flags;              /* B2P_EPI_C16_FP16: C16 holds fp16 (not bf16) bits               */
  uint64_t drop_seed;
  const float* residual;      /* optional: added last                                          */
  int64_t ldr, rbs1, rbs2;
  uint16_t* C16;              /* optional bf16 copy of the final value (strides of C); C may be
                               * NULL when only the bf16 copy is wanted (then beta must be 0)    */
  /* bf16 LDS-DMA kernel only (both operands bf16), nz1*nz2 == 1, no split-K:                   */
  uint16_t* pre16;            /* optional bf16 pre-activation store (instead of pre_out)       */
  const uint16_t* aux16;      /* act_bwd operand in bf16 (instead of aux; strides of aux)      */
  float* colsum_part;         /* optional: column sums of the final value per 32 output rows,
                               * [ceil(M/32)][N] floats (fused bias gradient; b2p_colsum_parts) */
  uint16_t* C16b;             /* optional second copy in bf16 beside an fp16 C16 (strides of C): the
                               * forward's fp16 operand and the backward's bf16 weight-gradient
                               * operand from one epilogue                                        */
} b2p_epilogue;

typedef struct {
  int64_t M, N, K;
  int32_t nz1, nz2;
  b2p_operand A, B;
  b2p_epilogue ep;
  int32_t precision;          /* 0 = bf16 MFMA, 1 = fp32 MFMA (parity mode), 2 = fp16 MFMA
                               * (fp32 operands converted while staged; forward of the 24-layer
                               * Conformer, whose CTC loss bf16 rounding noise biases), 3 = split
                               * bf16 (fp32 operands only: x = hi + lo, hi*hi + hi*lo + lo*hi on bf16
                               * MFMA, ~16 significant bits per product; the bf16x3 mode)       */
  int32_t timing_family;      /* tag for b2p_timing_* (0 = untagged)                          */
  double flops;               /* algorithmic FLOPs of this launch (for timing)                */
  /* split-K (deterministic): ksplit > 1 slices K into kchunk-sized ranges (multiple of 32) whose
   * fp32 partials go to workspace (>= ksplit*nz1*nz2*M*N floats) and are summed in slice order by
   * a reduce kernel; epilogue limited to alpha/beta. For under-filled grids (weight gradients). */
  int32_t ksplit, kchunk;
  float* workspace;
  int64_t workspace_floats;
} b2p_gemm_desc;

int b2p_gemm(const b2p_gemm_desc* d, b2p_stream_t stream);

/* ------------------------------------------------------------------ graph-replayed steps
 * A training step captured once as a HIP graph (train/step_graph.py) replays with host values
 * frozen. Dropout: every kernel adds (*dev_counter) * 0x9E3779B97F4A7C15 to its host-drawn seed
 * when a counter is set (NULL restores eager semantics); b2p_seed_epoch_step increments it (the
 * captured step's first node), so each replay draws new masks. */
int b2p_set_seed_epoch(const uint64_t* dev_counter);
/* LayerDrop gate (TF w2v / TF conf encoder LayerDrop inside a captured step): every GEMM and fused-
 * attention launch issued while a gate is set reads the device int *dev_flag when it runs; 0 skips
 * the GEMM's K loop (accumulators stay 0, the epilogue still writes finite outputs) and the
 * attention work (its backward writes zero gradients). NULL: ungated (default). */
int b2p_set_gate(const int32_t* dev_flag);
/* *flag = keep (1) / skip (0) of one layer for this replay: the draw b2p_layerdrop_select makes for
 * the same (p, seed) (step counter of b2p_set_seed_epoch mixed in). */
int b2p_layerdrop_flag(int32_t* flag, float p, uint64_t seed, b2p_stream_t stream);
int b2p_seed_epoch_step(uint64_t* dev_counter, b2p_stream_t stream);

/* ------------------------------------------------------------------ elementwise / reductions */
/* column sums over rows: out[n] (+)= sum_m X[m*ld + n]; used for bias grads. partial must hold
 * ceil(M/rows_per_block)*N floats (see b2p_colsum_workspace). */
int64_t b2p_colsum_workspace(int64_t M, int64_t N);
int b2p_colsum(const float* X, int64_t M, int64_t N, int64_t ld, float* out, int accumulate,
               float* partial, b2p_stream_t stream);
/* batched variant: out[b][n] (+)= sum_m f(X[b*bstride + m*ld + n]); mode 0: x, 1: x^2, 2: x*Y */
int b2p_colsum_batched(const float* X, const float* Y, int64_t batch, int64_t M, int64_t N, int64_t ld,
                       int64_t bstride, int mode, float* out, int accumulate, float* partial,
                       b2p_stream_t stream);

/* One-launch column sums take their arrival counters from a device pool, a fresh range per launch.
 * The ranges allocated between b2p_colsum_pin_begin and b2p_colsum_pin_end (a graph capture: the graph
 * replays those launches for as long as it lives) stay reserved until b2p_colsum_unpin(id); no later
 * launch is handed a reserved counter (when nothing free fits, it takes the two-launch form).
 * b2p_colsum_pool_state: the allocation cursor (set_cursor >= 0 moves it: tests) and the reserved
 * counter count. Replaces nothing in the reference (bookkeeping of the fused bias-gradient sums). */
/* bf16x3 mode: the split-bf16 image of an R x C fp32 operand (hi = bf16(x), lo = bf16(x - hi)) as three
 * blocks, block b = lo when bit b of pattern is set (A: hi, lo, hi = 0b010; B: hi, hi, lo = 0b100), side
 * by side per row (along_cols, ldy >= 3C) or stacked (ldy >= C): one bf16 GEMM over K' = 3K then sums
 * hi*hi + lo*hi + hi*lo (replaces the reference's fp32 matmuls at ~16 significant bits per product).
 * pattern | 16: two blocks (bits 0-1; ldy >= 2C side by side): the two-term images (hi, lo) . (hi, hi). */
int b2p_split3_bf16(const float* x, int64_t R, int64_t C, int64_t ldx, uint16_t* y, int64_t ldy, int pattern,
                    int along_cols, b2p_stream_t stream);
/* Per-member LayerDrop gates of a batched GEMM launch (nz1 members; the frozen weight gradients of several
 * layers in one launch): dev_gate_ptrs = device int64[nz1] of device int32* flags (0 = open), NULL to
 * clear; while set, b2p_gemm gates member z1 by its own flag instead of b2p_set_gate's. */
int b2p_set_gate_batch(const int64_t* dev_gate_ptrs);
/* dst[0 .. n) = vals[0 .. n), n <= 64, by a kernel launch carrying the values (graph-capturable): the
 * pointer / offset tables of batched launches. */
int b2p_i64_fill(int64_t* dst, const int64_t* vals, int n, b2p_stream_t stream);
/* Variant knob of the 16-bit GEMM launches (A/B tools, default from B2P_GEMM16_VARIANT), bits: 1 = the
 * 256-column ping-pong kernel without the quarter-scheduled operand DMA, 2 = no narrow (PBM x 128) ping-pong
 * kernel; v < 0 only reads. Returns the previous value. */
int b2p_gemm16_variant(int v);
int b2p_colsum_pin_begin(void);
int64_t b2p_colsum_pin_end(void);
int b2p_colsum_unpin(int64_t id);
int64_t b2p_colsum_pool_state(int64_t set_cursor, int64_t* reserved);
/* out[n] (+)= sum_t part[t][n] over ntiles rows of a b2p_epilogue.colsum_part buffer */
int b2p_colsum_parts(const float* part, int64_t ntiles, int64_t N, float* out, int accumulate,
                     b2p_stream_t stream);

/* dropout (forward and backward use the same mask): y = x * keep(seed, i) / (1-p) */
int b2p_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, b2p_stream_t stream);

/* LayerNorm over the last dim (transformers Wav2Vec2EncoderLayer.layer_norm / final_layer_norm,
 * Wav2Vec2Encoder.layer_norm; eps 1e-5). mean/rstd saved for backward. */
int b2p_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y,
                      float* mean, float* rstd, int64_t rows, int64_t cols, float eps,
                      float drop_p, uint64_t drop_seed, b2p_stream_t stream);
int64_t b2p_layernorm_bwd_workspace(int64_t rows, int64_t cols);
/* dy is the gradient of the (optionally dropped-out, drop_p/drop_seed) LN output; dx (+)= dx_accum.
 * If dx_dropped != NULL it also receives dx * mask(in_drop_seed)/(1-in_drop_p): the gradient of
 * the residual-branch dropout whose output fed this LayerNorm (post-LN encoder layers), and, if
 * dbias_in != NULL, its column sums (= the bias gradient of the Linear feeding that dropout). */
int b2p_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                      const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                      int64_t cols, const float* dx_accum, float drop_p, uint64_t drop_seed,
                      float* dx_dropped, float in_drop_p, uint64_t in_drop_seed, float* dbias_in,
                      float* workspace, b2p_stream_t stream);
/* As above, plus bf16 copies for the next GEMM's operand (NULL = none): y16 = bf16(y);
 * d16 = bf16(dx_dropped) when dx_dropped != NULL, else bf16(dx). */
int b2p_layernorm_fwd16(const float* x, const float* gamma, const float* beta, float* y, uint16_t* y16,
                        float* mean, float* rstd, int64_t rows, int64_t cols, float eps,
                        float drop_p, uint64_t drop_seed, b2p_stream_t stream);
int b2p_layernorm_bwd16(const float* dy, const float* x, const float* gamma, const float* mean,
                        const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                        int64_t cols, const float* dx_accum, float drop_p, uint64_t drop_seed,
                        float* dx_dropped, float in_drop_p, uint64_t in_drop_seed, float* dbias_in,
                        uint16_t* d16, float* workspace, b2p_stream_t stream);
/* b2p_layernorm_bwd16 with a second accumulator added to dx alone, after dx_accum and after the
 * dx_dropped / dbias_in outputs are formed (NULL = none; d16 of dx includes it): the skip-path
 * gradient of a LayerDrop-selected encoder layer (functional.layerdrop_layer), folded into the layer's
 * input-gradient LayerNorm instead of a separate add. With dgamma = dbeta = dbias_in = NULL the
 * parameter gradients are left as per-block partials in workspace: [3][nblk][cols] floats at offset
 * 0, nblk = ceil(rows / 16) (dgamma | dbeta | dbias_in rows, summed later by the caller). */
int b2p_layernorm_bwd_acc2(const float* dy, const float* x, const float* gamma, const float* mean,
                           const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                           int64_t cols, const float* dx_accum, const float* dx_accum2, float drop_p,
                           uint64_t drop_seed, float* dx_dropped, float in_drop_p, uint64_t in_drop_seed,
                           float* dbias_in, uint16_t* d16, float* workspace, b2p_stream_t stream);

/* fp32 -> bf16 (round to nearest even), the GEMM operand copy of a weight or activation
 * (master copies stay fp32; replaces the implicit .to(bfloat16) of autocast) */
int b2p_cast_bf16(const float* x, uint16_t* y, int64_t n, b2p_stream_t stream);
/* y[r][c] = 16-bit(x[r][c]) for an R x C block of a row-major fp32 matrix (row stride ldx) into a
 * 16-bit matrix of row stride ldy; fp16 = 0: bf16, 1: fp16 (both round-to-nearest-even, the
 * conversion the fp32-operand GEMM applies while staging). Stages fp32 GEMM operands for the
 * 16-bit LDS-DMA kernel (b2p_operand.dtype 1 / 2). */
int b2p_cast16_2d(const float* x, int64_t R, int64_t C, int64_t ldx, uint16_t* y, int64_t ldy, int fp16,
                  b2p_stream_t stream);
/* y[c * ldy + col0 + r] = bf16(x[r * C + c]): transposed bf16 copy of an R x C fp32 matrix (cached
 * k-contiguous weight operands of the backward-data GEMMs) */
int b2p_transpose_bf16(const float* x, uint16_t* y, int64_t R, int64_t C, int64_t ldy, int64_t col0,
                       b2p_stream_t stream);

/* Row softmax for attention scores (eager_attention_forward: softmax(QK^T*scale) + dropout).
 * S rows of length n (row stride ld). Writes P (pre-dropout) and Pd (dropped, scaled); the keep
 * mask of element (row, c) is b2p_keep(seed, row * (n rounded up to even) + c). */
int b2p_softmax_fwd(const float* S, float* P, float* Pd, int64_t rows, int64_t n, int64_t ld,
                    float drop_p, uint64_t drop_seed, b2p_stream_t stream);
/* dS = P * (dPd*mask - rowsum(P * dPd*mask)) */
int b2p_softmax_bwd(const float* P, const float* dPd, float* dS, int64_t rows, int64_t n,
                    int64_t ld, float drop_p, uint64_t drop_seed, b2p_stream_t stream);

/* elementwise activation backward: dx = dy * act'(pre) (optionally after dropout of dy) */
int b2p_act_bwd(const float* dy, const float* pre, float* dx, int64_t n, int act,
                b2p_stream_t stream);

/* ------------------------------------------------------------------ front-end
 * GaussianSmoothing (src/model/b2p2t_model.py:27-90): depthwise conv1d over time, taps[ntaps],
 * padding "same" (left (ntaps-1)/2, right ntaps/2) on x (B, L, C) channels-last. */
int b2p_gauss_smooth(const float* x, const float* taps, int ntaps, float* y, int64_t B,
                     int64_t L, int64_t C, b2p_stream_t stream);
/* col2im for Unfold((k,1), stride s) (src/model/b2p2t_model.py:108-113, 162-167) in tap-major
 * order: dX[b,l,c] = sum_{tap} dA[b, (l-tap)/s, tap*C + c], then (optionally) multiplied by
 * softsign'(Z[b,l,c]) (src/model/b2p2t_model.py:159). */
int b2p_unfold_col2im(const float* dA, const float* Z, float* dX, int64_t B, int64_t L,
                      int64_t C, int64_t T, int ktaps, int stride, b2p_stream_t stream);
/* day-weight gradient reduction: dW[d] = sum_{b: day[b]==d} dWb[b] (deterministic) */
int b2p_day_reduce(const float* per_sample, const int64_t* day_idx, int64_t B, int64_t ndays,
                   int64_t elems, float* out, b2p_stream_t stream);

/* ------------------------------------------------------------------ layout transforms */
/* Unfold((k,1), stride) of x (B, L, C) materialised tap-major in bf16: U[(b,t)][tap*C + c] =
 * bf16(x[b][t*stride + tap][c]), T = (L-k)/stride + 1 (b2p2t_model.py:108-113,162-167). bf16
 * mode's GRU layer-0 projection and weight-gradient operand. */
int b2p_unfold16(const float* x, uint16_t* U, int64_t B, int64_t L, int64_t C, int64_t k,
                 int64_t stride, b2p_stream_t stream);
/* Implicit-Unfold operands (L % s == 0, k % s == 0; functional._GRULayer): the Unfold of x (B, L, C)
 * is the overlapping-row view of a 16-bit copy of x (row stride s*C), never materialised; the input
 * gradient of the layer-0 projection is one GEMM over the overlapping-row view of the padded dgi
 * (b2p_pad_rows16) and the weight copy wb, with no (B*T, k*C) intermediate or col2im.
 * Replaces nn.Unfold((k,1), stride) + nn.GRU's layer-0 input projection (src/model/b2p2t_model.py:
 * 108-113, 162-167; src/model/brain_feature_extractor.py:39-47, 61-65) and their autograd.
 *  b2p_unfold_weight16: rows of w0 (G x C*k, reference layout [n][c*k + tap]) then w1 (may be NULL):
 *    wf[n][tap*C + c] (fp16 when fp16 = 1, else bf16; forward B operand) and, when wb != NULL,
 *    wb[j*Ntot + n][r*C + c] = bf16(w[n][c*k + s*(k/s-1-j) + r]), j < k/s, Ntot = rows of w0 + w1.
 *  b2p_pad_rows16: dst (lead + B*R rows of N) bf16: row lead + b*R + t = src[b][t] (src (B, T, N)
 *    fp32) for t < T, all other rows 0.
 *  b2p_cast16_tail: y[i] = 16-bit(x[i]) for i < n, 0 up to n_total (the tail an overlapping-row view
 *    reads past the last sample). */
int b2p_unfold_weight16(const float* w0, const float* w1, int64_t G, int64_t C, int64_t k, int64_t stride,
                        uint16_t* wf, int fp16, uint16_t* wb, b2p_stream_t stream);
int b2p_pad_rows16(const float* src, uint16_t* dst, int64_t B, int64_t T, int64_t N, int64_t R, int64_t lead,
                   b2p_stream_t stream);
int b2p_cast16_tail(const float* x, uint16_t* y, int64_t n, int64_t n_total, int fp16, b2p_stream_t stream);
/* records {dst, a, b, count} (int64 each; a / b may be 0 = NULL): dst[i] = a[i] + b[i] (fp32), all
 * records in one launch: the per-step assembly of stacked / concatenated small parameter tensors
 * (nn.GRU W_hh of both directions, b_ih + b_hh folds; src/model/brain_feature_extractor.py:39-47) */
int b2p_gather_recs(const int64_t* recs, int nrec, b2p_stream_t stream);
/* out[o][tap*I + i] = in[o][i*ntaps + tap]   (conv weight (O, I, taps) -> tap-major GEMM B)
 * inverse=1 does the opposite mapping; flip=1 reads tap (ntaps-1-tap). */
int b2p_conv_weight_permute(const float* in, float* out, int64_t O, int64_t I, int64_t ntaps,
                            int inverse, b2p_stream_t stream);
/* grouped conv-transpose weight: out[g][i][k'*Og + o] = w[(g*Og+o)][i][ntaps-1-k'] and inverse */
int b2p_conv_weight_transpose_flip(const float* w, float* out, int64_t G, int64_t Og, int64_t I,
                                   int64_t ntaps, b2p_stream_t stream);

/* weight norm over all dims but dim=2 (torch.nn.utils.parametrizations.weight_norm(dim=2),
 * transformers Wav2Vec2PositionalConvEmbedding): w[o,i,k] = g[k] * v[o,i,k] / ||v[:,:,k]|| */
/* Greedy CTC decode + word errors of a batch on the device (replaces the train
 * evaluator's host round trip, src/train/evaluator.py:69-129): argmax per frame (first maximum),
 * group repeats, drop `blank`, cut after the first `eos`; words split at `delim`; per sample the
 * word-level Levenshtein distance to the target (pads dropped) and the target's word count
 * (WER = sum errs / sum nwords). out_tokens [B][T] int32 (first out_ntok[b] valid). T <= 1024. */
int b2p_ctc_greedy_wer(const float* logits, int64_t B, int64_t T, int64_t C, const int64_t* target, int64_t S,
                       int blank, int eos, int delim, int32_t* out_tokens, int32_t* out_ntok, int32_t* errs,
                       int32_t* nwords, b2p_stream_t stream);
/* Character errors of the same greedy decode (reference EvaluatorWithW2vLMDecoder
 * .calculate_char_error_rate, src/train/evaluator.py:212-214,231-242): prediction and target
 * rendered to characters as Wav2Vec2CTCTokenizer.batch_decode does (token id -> tok_chars[id*8 ..
 * +tok_len[id]), delim -> ' ', stripped, prediction cut after the first eos), per-sample
 * Levenshtein distance char_errs[b] and target length nchars[b] (CER = sum errs / sum nchars).
 * char_errs[b] = -1 if a rendered string exceeds 2048 characters. */
int b2p_ctc_greedy_cer(const float* logits, int64_t B, int64_t T, int64_t C, const int64_t* target, int64_t S,
                       int blank, int eos, int delim, const uint8_t* tok_chars, const int32_t* tok_len,
                       int32_t* char_errs, int32_t* nchars, b2p_stream_t stream);
/* CTC prefix beam search without a language model (csrc/beam.hip; the LM-free part of the
 * reference's pyctcdecode test decode, src/train/evaluator.py:189-210): logits (B, T, C) raw scores
 * (log-softmax applied per frame), lens (B) frames to decode per sample (NULL: T), beam width
 * <= 128, C <= 64; characters below token_min_logp are skipped unless they are the frame's argmax,
 * candidates below best + beam_prune_logp dropped. workspace: b2p_ctc_beam_workspace(B, T, beam)
 * int32. Outputs: out_tokens (B, T) collapsed token ids of the best prefix (-1 padded), out_len (B),
 * out_score (B) its log probability (log p_b + p_nb). */
int64_t b2p_ctc_beam_workspace(int64_t B, int64_t T, int64_t beam);
int b2p_ctc_prefix_beam(const float* logits, int64_t B, int64_t T, int64_t C, const int32_t* lens, int64_t beam,
                        int blank, float token_min_logp, float beam_prune_logp, int32_t* workspace,
                        int32_t* out_tokens, int32_t* out_len, float* out_score, b2p_stream_t stream);

/* Grouped positional conv of wav2vec2 on bf16 MFMA (csrc/posconv16.hip; 48 channels per group,
 * 128 taps, padding 64 + SamePad, T <= 256), replacing the implicit-conv GEMMs of
 * Wav2Vec2PositionalConvEmbedding (modeling_wav2vec2.py, reached from
 * src/model/w2v_custom_feat_extractor.py:152 through the encoder):
 *   fwd:       pre = conv(e) + bias, xsum = gelu(pre) + e, e16 = bf16(e); w16 = bf16 [O][taps*Ig]
 *              (b2p_conv_weight_permute layout)
 *   bwd_data:  dpre = dxsum * gelu'(pre), de = conv^T(dpre) + dxsum, dpre16 = bf16(dpre),
 *              colpart[b][c] = sum_t dpre[b,t,c]; wt16 = bf16 b2p_conv_weight_transpose_flip layout
 *   wgrad:     dwp[o][tap*Ig + i] = sum_{b,t} dpre[b,t,o] * e[b,t+tap-64,i] (bf16 operands, fp32 sums) */
int b2p_posconv16_fwd(const float* e, const uint16_t* w16, const float* bias, float* xsum, float* pre,
                      uint16_t* e16, int64_t B, int64_t T, int64_t D, int64_t groups, b2p_stream_t stream);
int b2p_posconv16_bwd_data(const float* dxsum, const float* pre, const uint16_t* wt16, float* de, uint16_t* dpre16,
                           float* colpart, int64_t B, int64_t T, int64_t D, int64_t groups, b2p_stream_t stream);
int b2p_posconv16_wgrad(const uint16_t* dpre16, const uint16_t* e16, float* dwp, int64_t B, int64_t T, int64_t D,
                        int64_t groups, b2p_stream_t stream);
int64_t b2p_weight_norm_workspace(int64_t O, int64_t I, int64_t K);
int b2p_weight_norm_fwd(const float* g, const float* v, float* w, float* norms, int64_t O,
                        int64_t I, int64_t K, float* workspace, b2p_stream_t stream);
int b2p_weight_norm_bwd(const float* g, const float* v, const float* norms, const float* dw,
                        float* dg, float* dv, int64_t O, int64_t I, int64_t K, float* workspace,
                        b2p_stream_t stream);

/* ------------------------------------------------------------------ GRU recurrence
 * nn.GRU (src/model/brain_feature_extractor.py:39-47, 56-68), PyTorch gate order (r,z,n),
 * bidirectional, batch_first, h0 = 0 (or h0 given). gi = x W_ih^T + b_ih precomputed by
 * b2p_gemm for both directions: gi[b][t][dir*3H + g*H + j]. whh: [2][3H][H], bhh: [2][3H].
 * Outputs: out[b][t][dir*H + j]; saved gates for backward: rzn [B][T][2][4][H]
 * (r, z, n, W_hn h + b_hn). */
int b2p_gru_fwd(const float* gi, const float* whh, const float* bhh, const float* h0,
                float* out, float* saved, int64_t B, int64_t T, int64_t H, int ndir,
                b2p_stream_t stream);
/* BPTT: dout [B][T][ndir*H] -> dgi [B][T][ndir*3H] (= dgh except the n-gate, also returned in
 * dgh [B][T][ndir*3H]) and, if dh0 != NULL, dh0 [ndir][B][H]. dhbuf: ndir*B*H floats scratch.
 * Weight grads are GEMMs on (dgh, h_prev), bias grads column sums. */
int b2p_gru_bwd(const float* dout, const float* whh, const float* out, const float* saved,
                const float* h0, float* dgi, float* dgh, float* dh0, float* dhbuf, int64_t B,
                int64_t T, int64_t H, int ndir, b2p_stream_t stream);
/* Persistent bf16-MFMA recurrence (bf16 precision mode; csrc/gru16.hip): one workgroup runs the
 * whole time loop of one direction for 16 batch rows with W_hh resident on the CU (registers +
 * LDS) — one launch per layer instead of one per time step (replaces the cuDNN RNN behind
 * nn.GRU, src/model/brain_feature_extractor.py:39-47). Per-step tensors are LANE-NATIVE ("LN"):
 * for direction d, 16-row batch group bg, processing step s (= t forward, T-1-t reverse),
 * 16-unit block ub and record r, float offset
 *   (((((d*NBG + bg)*T + s)*(H/16) + ub)*R + r)*64 + lane)*4 + i,
 *   lane = b%16 + 16*((j%16)/4), i = j%4   (NBG = ceil(B/16); b2p_gru16_lane_floats sizes it).
 * fwd: giL = LN(R=3) of x W_ih^T + b_ih + [b_hr, b_hz, 0] (b_hh's r/z parts folded in; bhh is
 *      read for b_hn only) -> hL = LN(R=1) of h, savL = LN(R=4) of (r, z, n, W_hn h + b_hn).
 * bwd: doL = LN(R=1) of dOut, hL/savL from fwd -> dgL = LN(R=4) of (dar, daz, dan, dan*r)
 *      (= dgi gates 0..2, dgh = records 0, 1, 3); dh0 [ndir][B][H] optional.
 * b2p_gru_lane_permute: standard (B, T, ndir*Rs*H) <-> LN(Rl); rmap nibble k = standard record of
 * LN record k (15 = skip), to_lane selects the direction. Supported H: b2p_gru16_supported(H) (32, 64, 128, 256). */
int b2p_gru16_supported(int64_t H);
int64_t b2p_gru16_lane_floats(int64_t B, int64_t T, int64_t H, int ndir, int R);
int b2p_gru_lane_permute(const float* src, float* dst, int64_t B, int64_t T, int64_t H, int ndir,
                         int Rl, int Rs, uint32_t rmap, int to_lane, b2p_stream_t stream);
int b2p_gru_fwd16(const float* giL, const float* whh, const float* bhh, const float* h0,
                  float* hL, float* savL, int64_t B, int64_t T, int64_t H, int ndir,
                  b2p_stream_t stream);
int b2p_gru_bwd16(const float* doL, const float* whh, const float* hL, const float* savL,
                  const float* h0, float* dgL, float* dh0, int64_t B, int64_t T, int64_t H,
                  int ndir, b2p_stream_t stream);
/* h_prev sequence for the weight-gradient GEMM: hp[dir][b][t][j] = h_{t-1} in that direction's
 * processing order (h0 at the first step). */
int b2p_gru_hprev(const float* out, const float* h0, float* hp, int64_t B, int64_t T, int64_t H,
                  int ndir, b2p_stream_t stream);

/* ------------------------------------------------------------------ multi-CU persistent GRU (bf16)
 * csrc/grumc.hip: the whole recurrence of an nn.GRU layer in one launch for hidden sizes one CU
 * cannot hold (256, 384, 512; the Conformer experiment's H = 512 encoder, reference
 * src/model/brain_feature_extractor.py:39-47). H/64 workgroups per (direction, 16 batch rows), each
 * keeping its units' W_hh rows in registers, exchange the state every step through L2 as tagged
 * granules. Same tensors and layouts as b2p_gru_fwd / b2p_gru_bwd (standard (B, T, ...) layouts);
 * bf16 MFMA operands, fp32 accumulation and state. workspace: b2p_gru_mc_workspace(B, H, ndir)
 * bytes, 16-byte aligned, zeroed by the call itself (the first int is a timeout flag: nonzero after
 * the call means a member never arrived; the second counts the recurrences whose members all ran
 * on one XCD and exchanged through its L2). Needs (H/64) * ndir * ceil(B/16) co-resident CUs. */
int b2p_gru_mc_supported(int64_t H);
int64_t b2p_gru_mc_workspace(int64_t B, int64_t H, int ndir);
int b2p_gru_fwd_mc(const float* gi, const float* whh, const float* bhh, const float* h0, float* out,
                   float* saved, void* workspace, int64_t B, int64_t T, int64_t H, int ndir,
                   b2p_stream_t stream);
int b2p_gru_bwd_mc(const float* dout, const float* whh, const float* out, const float* saved,
                   const float* h0, float* dgi, float* dgh, float* dh0, void* workspace, int64_t B,
                   int64_t T, int64_t H, int ndir, b2p_stream_t stream);   /* T + 1 <= 65535 (16-bit tag) */
/* Stream-ordered after a b2p_gru_fwd_mc / b2p_gru_bwd_mc call on `workspace`: if that launch timed
 * out, *status = code unless *status is already nonzero (the first failure is kept). status is a
 * persistent device int32 the caller zeroes once and reads at its next host sync (the Python layer
 * raises RuntimeError naming the recurrence; functional.check_gru_status). Capturable. */
int b2p_gru_mc_status(const void* workspace, int32_t* status, int32_t code, b2p_stream_t stream);
/* test knob: member `member` (0..15) of every recurrence skips its state exchange stores from the
 * next launch on, so the other members time out (-1: off) */
int b2p_gru_mc_debug_withhold(int member);

/* ------------------------------------------------------------------ fused attention (bf16 mode)
 * softmax(Q K^T * scale) -> dropout(p) -> @ V per (batch, head), no mask (HF Wav2Vec2Attention,
 * TF w2v:438-463,529-545; the Conformer's rotary self-attention core, TF conf:458-470);
 * csrc/attn16.hip. Head size 64, T <= 256 (whole K/V of a head in LDS, scores never in HBM).
 * qkv16: bf16 [B*T][3*nh*64] (q | k | v, head-major), O16: bf16 [B*T][nh*64], lse2: f32 [B][nh][T]
 * (row max + log2 sum of the log2e-scaled scores, saved for backward). Dropout keep mask =
 * b2p_keep(seed, ((b*nh + h)*T + q)*TP + key), TP = T rounded up to even (B*nh*T*TP < 2^32),
 * identical to b2p_softmax_fwd's. fwd runs one workgroup per (batch, head, 128 queries). bwd writes
 * [dQ | dK | dV] into dqkv (f32, may be NULL) and/or dqkv16 (bf16, may be NULL), same layout as qkv;
 * delta_ws: B*nh*T floats of workspace (row constants sum_key P_d dP_d). mask (optional, drop_p > 0):
 * 32 bytes per query row ([B][nh][T][32] uint8), written by fwd and read by bwd instead of re-hashing
 * every (q, key) twice: byte 8*g + c with g = (key >> 2) & 3 and c = key >> 5 holds keys 32c + 4g + i
 * (bit i) and 32c + 16 + 4g + i (bit 4 + i), i < 4 (each forward lane writes its own 8 bytes);
 * NULL: bwd recomputes the hash. */
int b2p_attn16_fwd(const void* qkv16, void* O16, float* lse2, int64_t B, int64_t T, int64_t nh,
                   int64_t dh, float scale, float drop_p, uint64_t drop_seed, uint32_t* mask,
                   b2p_stream_t stream);
/* fp16-operand forward (the bf16 precision mode's attention operands: 11 significant bits for Q, K, V and
 * the probabilities instead of bf16's 8; same rate): qkv16h and O16h hold fp16 bits, Ob16 (may be NULL)
 * receives a bf16 copy of O for the out-projection's weight gradient. The backward of such a forward is
 * b2p_attn16_bwd_f16. */
int b2p_attn16_fwd_f16(const void* qkv16h, void* O16h, void* Ob16, float* lse2, int64_t B, int64_t T,
                       int64_t nh, int64_t dh, float scale, float drop_p, uint64_t drop_seed, uint32_t* mask,
                       b2p_stream_t stream);
/* Dropout keep bits of n_layers attention launches drawn ahead in one launch: mask (n_layers, B, nh, T, 8)
 * int32, layer l's block equal word for word to the mask b2p_attn16_fwd[_f16] stores with seed seeds[l]
 * (a host array; the graph-replay step counter is mixed in as there). T <= 256, 0 < drop_p < 1. Replaces
 * the per-layer draw inside the reference's attention dropout (TF w2v Wav2Vec2Attention.forward
 * nn.functional.dropout(attn_weights), TF conf :458-470); the encoder issues it beside the GRU. */
int b2p_attn16_keep_masks(uint32_t* mask, const uint64_t* seeds, int64_t n_layers, int64_t B, int64_t T,
                          int64_t nh, float drop_p, b2p_stream_t stream);
/* b2p_attn16_fwd / b2p_attn16_fwd_f16 with the keep bits READ from mask (one layer's block of
 * b2p_attn16_keep_masks, or a mask an earlier forward stored): same outputs as the storing forward with
 * that mask's seed; the backward takes the same mask. */
int b2p_attn16_fwd_keep(const void* qkv16, void* O16, float* lse2, int64_t B, int64_t T, int64_t nh,
                        int64_t dh, float scale, float drop_p, const uint32_t* mask, b2p_stream_t stream);
int b2p_attn16_fwd_f16_keep(const void* qkv16h, void* O16h, void* Ob16, float* lse2, int64_t B, int64_t T,
                            int64_t nh, int64_t dh, float scale, float drop_p, const uint32_t* mask,
                            b2p_stream_t stream);
int b2p_attn16_bwd(const void* qkv16, const void* dO16, const float* lse2, float* delta_ws,
                   float* dqkv, void* dqkv16, int64_t B, int64_t T, int64_t nh, int64_t dh,
                   float scale, float drop_p, uint64_t drop_seed, const uint32_t* mask, b2p_stream_t stream);
/* backward of b2p_attn16_fwd_f16: qkv16h fp16. The scores are recomputed on fp16 MFMA from the same
 * operands as the forward (consistent with its lse2, so saturated softmax rows give ~0 dS as in fp32);
 * the products with the bf16 gradients (dP = dO V^T, dQ = dS K, dK = dS^T Q) take bf16 conversions of
 * V, K, Q made in registers / while staging LDS. Same outputs and workspace as b2p_attn16_bwd. */
int b2p_attn16_bwd_f16(const void* qkv16h, const void* dO16, const float* lse2, float* delta_ws,
                       float* dqkv, void* dqkv16, int64_t B, int64_t T, int64_t nh, int64_t dh,
                       float scale, float drop_p, uint64_t drop_seed, const uint32_t* mask, b2p_stream_t stream);
/* Selects the dK/dV kernel of b2p_attn16_bwd[_f16]: 1 (default) = each wave runs its two key tiles in
 * one pass over the queries (shared LDS reads and conversions), 0 = one pass per key tile. Both
 * accumulate in the same order, so the outputs are bitwise equal. Process-wide; the initial value
 * comes from B2P_ATTN_DKV2 (0 selects the per-tile kernel). */
int b2p_attn16_dkv_variant(int v);

/* ------------------------------------------------------------------ CTC
 * log_softmax + nn.CTCLoss(blank=0, reduction="mean", zero_infinity=True)
 * (src/model/w2v_custom_feat_extractor.py:59, 81-90). logits (B, T, C) batch-first; targets
 * (B, S) int64 (entries beyond target_len ignored); in_lens int32 (B), tgt_lens int64 (B).
 * Writes per-sample nll (B; +inf when infeasible), the mean loss (1; infeasible samples count
 * as 0 = zero_infinity), and grad_logits (B, T, C) = d(mean loss)/d(logits) (zero for
 * t >= in_len and for infeasible samples). Workspace: b2p_ctc_workspace floats. */
int64_t b2p_ctc_workspace(int64_t B, int64_t T, int64_t S, int64_t C);
int b2p_ctc_fwd_bwd(const float* logits, const int64_t* targets, const int32_t* in_lens,
                    const int64_t* tgt_lens, int64_t B, int64_t T, int64_t S, int64_t C,
                    int blank, float* nll, float* loss, float* grad_logits, float* workspace,
                    b2p_stream_t stream);

/* ------------------------------------------------------------------ Adam
 * torch.optim.Adam (src/experiments/experiment.py:25-28, b2t_gru_w2v_experiment.py:138-145):
 * L2 weight decay, bias correction, eps outside the sqrt. Multi-tensor: `table` is a device
 * array of ntensors records {param*, grad*, exp_avg*, exp_avg_sq*, numel} (5 x int64). */
int b2p_adam_multi(const int64_t* table, int ntensors, int64_t max_numel, float lr, float beta1,
                   float beta2, float eps, float weight_decay, float bias_c1, float bias_c2_sqrt,
                   b2p_stream_t stream);
/* the same update with lr read from lr_dev[0] and the step counter step_dev[0] (double) incremented
 * and turned into the bias corrections on the device (hyper_dev: float[3] scratch): replayable in a
 * captured step (torch.optim.Adam capturable=True semantics) */
int b2p_adam_multi_dev(const int64_t* table, int ntensors, int64_t max_numel, const float* lr_dev, float beta1,
                       float beta2, float eps, float weight_decay, double* step_dev, float* hyper_dev,
                       b2p_stream_t stream);
/* the update with the tensor records {param, grad, exp_avg, exp_avg_sq, numel} read from HOST
 * memory by the launcher and passed in the kernel arguments (48 tensors per launch): no device
 * table to upload, so it is also capturable. step_dev == NULL: host lr / bias corrections;
 * otherwise the device form of b2p_adam_multi_dev, its bias corrections formed in double from the
 * double betas exactly as the host computes them for torch.optim.Adam. */
int b2p_adam_recs(const int64_t* recs, int ntensors, float lr, double beta1, double beta2, float eps,
                  float weight_decay, float bias_c1, float bias_c2_sqrt, const float* lr_dev, double* step_dev,
                  float* hyper_dev, b2p_stream_t stream);
/* Per-tensor device step counters and gates (HipAdam's device form, used in captured and in data-
 * parallel steps). torch.optim.Adam skips a parameter whose .grad is None: no moment update, no
 * weight decay, no step increment (src/experiments/experiment.py:25-28); under LayerDrop the
 * reference's skipped encoder layers are such parameters. Records of 7 x int64 read from HOST memory
 * (32 per launch pair, capturable): {param, grad, exp_avg, exp_avg_sq, numel, step (double*, that
 * tensor's counter), gate (int32*: 0 = skip this tensor; NULL = always update)}. lr from lr_dev[0];
 * the bias corrections are formed per tensor in double from its own step and rounded to float, as
 * the host form (b2p_adam_recs) receives them, and the element update is the same code: both forms
 * are bit-identical for equal inputs. hyper_dev: float[4 * ntensors] scratch (16-B aligned). */
int b2p_adam_gated_recs(const int64_t* recs, int ntensors, const float* lr_dev, double beta1, double beta2,
                        float eps, float weight_decay, float* hyper_dev, b2p_stream_t stream);

/* dst += src (fp32) for ntensors records {dst, src, numel} read from HOST memory and passed in the
 * kernel arguments (96 per launch; capturable): the per-step accumulation of the small gradients of
 * frozen parameters into their .grad (src/train/train_loop.py:44,66 never zeroes them), one launch
 * instead of one elementwise add per tensor. */
int b2p_accum_recs(const int64_t* recs, int ntensors, b2p_stream_t stream);
/* row-summing form: records {dst, src, numel, nrows, set} (5 x int64 each):
 * dst[i] (set ? = : +=) sum_{r < nrows} src[r * numel + i], rows summed in order (nrows >= 1). Takes
 * column sums still held as per-tile partial rows (b2p_gemm colsum_part, b2p_drop_cast_colsum) and
 * finishes them inside the batched accumulation (replaces b2p_colsum_parts + the add); reference: the
 * bias gradients torch autograd accumulates into .grad (TF w2v / conf Linear layers). */
int b2p_accum_rows_recs(const int64_t* recs, int ntensors, b2p_stream_t stream);

/* dropout with an extra output scale: y = x * keep(seed, i) * scale / (1-p) (macaron half-step) */
/* out_lens[i] = (int32)((float)(in_lens[i] - kernel) / (float)stride): the unfolded input lengths of
 * src/model/b2p2t_model.py:170-173 (int64 lengths, float32 true division, truncation), one launch. */
int b2p_unfold_lens(const int64_t* in_lens, int32_t* out_lens, int64_t n, int64_t kernel, int64_t stride,
                    b2p_stream_t stream);
/* out[i] = targets[i] < 1 ? -100 : targets[i] (int64): the CTC targets of
 * src/model/w2v_custom_feat_extractor.py:70 / w2v_conformer_custom_feat_extractor.py:41, one launch. */
int b2p_ctc_targets(const int64_t* targets, int64_t* out, int64_t n, b2p_stream_t stream);
/* y = x * (*s) with the scalar s read on the device (16-B aligned x, y): the CTC loss backward's
 * grad * grad_output (torch.autograd seeds a reduced loss with a device scalar). */
int b2p_scale_by_device_scalar(const float* x, const float* s, float* y, int64_t n, b2p_stream_t stream);
int b2p_dropout_scaled(const float* x, float* y, int64_t n, float p, uint64_t seed, float scale,
                       b2p_stream_t stream);
/* Output-dropout backward of a Conformer block in one pass (replaces b2p_dropout_scaled + a bf16
 * cast + b2p_colsum of its result; reference TF conf Wav2Vec2ConformerFeedForward / SelfAttention /
 * ConvolutionModule output dropout): y16 = bf16(mask(x) * scale / (1 - p)) over M x N (N % 4 == 0),
 * and when part != NULL the per-64-row column partial sums of those fp32 values,
 * part[b2p_drop_cast_colsum_parts(M)][N] (finish with b2p_colsum_parts). Same mask as
 * b2p_dropout_scaled. */
int64_t b2p_drop_cast_colsum_parts(int64_t M);
int b2p_drop_cast_colsum(const float* x, uint16_t* y16, float* part, int64_t M, int64_t N, float p, uint64_t seed,
                         float scale, b2p_stream_t stream);
/* LayerNorm forward (TF conf / TF w2v nn.LayerNorm) writing the 16-bit GEMM operand copy y16 (fp16 when
 * y16_fp16, else bf16) and optionally a bf16 copy y16b (the backward's weight-gradient operand);
 * y (fp32) may be NULL. No dropout. */
int b2p_layernorm_fwd_x16(const float* x, const float* gamma, const float* beta, float* y, uint16_t* y16, int y16_fp16,
                          uint16_t* y16b, float* mean, float* rstd, int64_t rows, int64_t cols, float eps,
                          b2p_stream_t stream);
/* Forward rotary embedding (as b2p_rotary, inverse 0) written as a 16-bit operand (fp16 when fp16). */
int b2p_rotary16(const float* x, const float* cos_t, const float* sin_t, uint16_t* out, int fp16, int64_t B, int64_t T,
                 int64_t H, int64_t D, int64_t ld, b2p_stream_t stream);
/* LayerNorm + rotary embedding in one pass for the Conformer attention block (TF conf
 * Wav2Vec2ConformerSelfAttention with position_embeddings_type="rotary": query and key read the rotated
 * LN output, value the plain one). 16-bit outputs only, each optional (NULL skips it): h16 / hr16 the
 * forward operands (fp16 when half16, else bf16), h16b / hr16b bf16 copies for the weight gradients.
 * Equal bit for bit to b2p_layernorm_fwd_x16 followed by b2p_rotary16 of the fp32 output.
 * cols % 256 == 0, cols <= 1024, head_dim in {32, 64, 128, 256}, rows = B * T. */
int b2p_layernorm_rotary16(const float* x, const float* gamma, const float* beta, float* mean, float* rstd,
                           int64_t rows, int64_t cols, float eps, int64_t T, int64_t head_dim, const float* cos_t,
                           const float* sin_t, int half16, uint16_t* h16, uint16_t* h16b, uint16_t* hr16,
                           uint16_t* hr16b, b2p_stream_t stream);
/* out = bf16(dropout(act(pre))) with the mask of a GEMM epilogue over the same flat index (n % 4 == 0):
 * recomputes a Conformer FFN intermediate (TF conf Wav2Vec2ConformerFeedForward) for its weight
 * gradient. */
int b2p_act_dropout_cast16(const float* pre, uint16_t* out, int64_t n, int act, float p, uint64_t seed,
                           b2p_stream_t stream);

/* ------------------------------------------------------------------ Conformer
 * transformers Wav2Vec2Conformer{SelfAttention,ConvolutionModule,RotaryPositionalEmbedding}
 * as instantiated by reference src/model/w2v_conformer_custom_feat_extractor.py:62-112. */
/* rotary on (B*T rows of H heads x D, row stride ld): out = x*cos + rotate_half(x)*sin with
 * rotate_half(x) = cat(-x2, x1); inverse=1 applies the transpose (backward). cos/sin (T, D). */
int b2p_rotary(const float* x, const float* cos_t, const float* sin_t, float* out, int64_t B,
               int64_t T, int64_t H, int64_t D, int64_t ld, int inverse, b2p_stream_t stream);
/* nn.GLU(dim=channels): out[m][c] = a[m][c] * sigmoid(a[m][C+c]); a is (M, 2C) */
int b2p_glu_fwd(const float* a, float* out, int64_t M, int64_t C, b2p_stream_t stream);
int b2p_glu_bwd(const float* a, const float* dout, float* da, int64_t M, int64_t C,
                b2p_stream_t stream);
/* GLU backward (TF conf Wav2Vec2ConformerConvolutionModule nn.GLU(dim=1)) written as the bf16 operand
 * of the pointwise-conv-1 backward GEMMs: da16 (M, 2C), C % 4 == 0. */
int b2p_glu_bwd16(const float* a, const float* dout, uint16_t* da16, int64_t M, int64_t C, b2p_stream_t stream);
/* depthwise Conv1d(C, C, K, padding=(K-1)/2, groups=C, bias=False), channels-last (B, T, C);
 * w (C, K). Backward writes dx and/or dw (deterministic partial sums). */
int b2p_dwconv_fwd(const float* x, const float* w, float* y, int64_t B, int64_t T, int64_t C,
                   int K, b2p_stream_t stream);
int64_t b2p_dwconv_bwd_workspace(int64_t B, int64_t T, int64_t C, int K);
int b2p_dwconv_bwd(const float* x, const float* w, const float* dy, float* dx, float* dw,
                   int64_t B, int64_t T, int64_t C, int K, float* workspace, b2p_stream_t stream);
/* BatchNorm1d over channels of (M, C) rows: training mode uses batch statistics (two-pass mean /
 * biased variance), updates running stats (momentum, unbiased variance), applies gamma/beta and the
 * fused activation act (B2P_ACT_SILU = swish). pre (optional) keeps the pre-activation. */
int64_t b2p_batchnorm_workspace(int64_t M, int64_t C);
/* num_batches_tracked (int64, device) of the next training-mode statistics launch on this host thread
 * (b2p_batchnorm_fwd, or b2p_batchnorm_finalize phase 1): that launch adds 1 to it on the device,
 * unless the LayerDrop gate (b2p_set_gate) is closed -- torch _BatchNorm.forward's
 * num_batches_tracked.add_(1) without a separate launch. NULL clears it. */
int b2p_batchnorm_count_next(int64_t* num_batches_tracked);
int b2p_batchnorm_fwd(const float* x, const float* gamma, const float* beta, float* running_mean,
                      float* running_var, float* y, float* pre, float* mean, float* rstd, int64_t M,
                      int64_t C, float eps, float momentum, int act, float* workspace,
                      b2p_stream_t stream);
int b2p_batchnorm_eval(const float* x, const float* gamma, const float* beta,
                       const float* running_mean, const float* running_var, float* y, int64_t M,
                       int64_t C, float eps, int act, float* workspace, b2p_stream_t stream);
int b2p_batchnorm_bwd(const float* dy, const float* pre, const float* x, const float* mean,
                      const float* rstd, const float* gamma, float* dx, float* dgamma, float* dbeta,
                      int64_t M, int64_t C, int act, float* workspace, b2p_stream_t stream);

/* BatchNorm in stages, for synchronised statistics across data-parallel ranks (SyncBN; SURVEY
 * 8(e3)(iii)): the caller all-reduces the per-channel sums between the stages.
 *   stats    : out[c] = sum_m x[m][c] (center NULL) or sum_m (x[m][c] - center[c])^2
 *   finalize : mean = sum / count (phase 0, in place on sum -> mean); phase 1: rstd from the summed
 *              squared deviations and the running-stat update (count = global row count)
 *   apply    : y = act(pre), pre = (x - mean) * rstd * gamma + beta
 *   bwd_sums : g = dy * act'(pre) (into g, M*C), sum_g[c], sum_gx[c] = sum g * xhat
 *   bwd_dx   : dx = gamma * rstd * (g - sum_g / count - xhat * sum_gx / count)
 * workspace: b2p_batchnorm_workspace(M, C) floats. */
int b2p_batchnorm_stats(const float* x, const float* center, float* out, int64_t M, int64_t C,
                        float* workspace, b2p_stream_t stream);
int b2p_batchnorm_finalize(float* sum_or_mean, const float* sqdev, float* rstd, float* running_mean,
                           float* running_var, int64_t C, int64_t count, float eps, float momentum,
                           int phase, b2p_stream_t stream);
int b2p_batchnorm_apply(const float* x, const float* mean, const float* rstd, const float* gamma,
                        const float* beta, float* y, float* pre, int64_t M, int64_t C, int act,
                        b2p_stream_t stream);
/* b2p_batchnorm_fwd / b2p_batchnorm_apply writing the activation output as 16-bit GEMM operands: y (fp32),
 * y16 (fp16 when y16_fp16, else bf16) and y16b (bf16) are each optional, at least one is given (TF conf
 * Wav2Vec2ConformerConvolutionModule: BN -> activation -> pointwise_conv2; the conv module keeps the
 * fp16 forward operand and the bf16 weight-gradient operand only). C % 4 == 0, aligned pointers. */
int b2p_batchnorm_fwd16(const float* x, const float* gamma, const float* beta, float* running_mean, float* running_var,
                        float* y, uint16_t* y16, int y16_fp16, uint16_t* y16b, float* pre, float* mean, float* rstd,
                        int64_t M, int64_t C, float eps, float momentum, int act, float* workspace,
                        b2p_stream_t stream);
int b2p_batchnorm_apply16(const float* x, const float* mean, const float* rstd, const float* gamma, const float* beta,
                          float* y, uint16_t* y16, int y16_fp16, uint16_t* y16b, float* pre, int64_t M, int64_t C,
                          int act, b2p_stream_t stream);
int b2p_batchnorm_bwd_sums(const float* dy, const float* pre, const float* x, const float* mean,
                           const float* rstd, float* g, float* sum_g, float* sum_gx, int64_t M,
                           int64_t C, int act, float* workspace, b2p_stream_t stream);
int b2p_batchnorm_bwd_dx(const float* g, const float* x, const float* mean, const float* rstd,
                         const float* gamma, const float* sum_g, const float* sum_gx, float* dx,
                         int64_t M, int64_t C, int64_t count, b2p_stream_t stream);

/* ------------------------------------------------------------------ LayerDrop in a captured step
 * (csrc/layerdrop.hip). The reference skips an encoder layer when torch.rand([]) < layerdrop (TF
 * w2v Wav2Vec2Encoder.forward, TF conf Wav2Vec2ConformerEncoder.forward), a host decision a
 * captured graph cannot redraw. In a graph every layer runs and the decision is drawn on the device,
 * keep = hash(seed + step counter) >= p, so each replay redraws it:
 *   select: out = keep ? keep_val : skip_val (and out16 from keep16/skip16 or a cast, if out16)
 *   route : d_keep = keep ? dout : 0, d_skip = keep ? 0 : dout
 *   keep  : the same draw on the host (epoch = the step counter's value, has_epoch 0 = eager). */
int b2p_layerdrop_keep(float p, uint64_t seed, uint64_t epoch, int has_epoch, int32_t* keep);
int b2p_layerdrop_select(const float* skip_val, const float* keep_val, float* out,
                         const uint16_t* skip16, const uint16_t* keep16, uint16_t* out16, int64_t n,
                         float p, uint64_t seed, b2p_stream_t stream);
/* b2p_layerdrop_select plus the fp16 copy (outh from skiph / keeph, or packed from the selected values
 * when the chosen one is NULL): the next post-LN layer's fp16 forward operand, so it needs no cast.
 * out == keep_val with out16 == keep16 and outh == keeph selects in place: a kept layer moves no bytes. */
int b2p_layerdrop_select_h(const float* skip_val, const float* keep_val, float* out, const uint16_t* skip16,
                           const uint16_t* keep16, uint16_t* out16, const uint16_t* skiph, const uint16_t* keeph,
                           uint16_t* outh, int64_t n, float p, uint64_t seed, b2p_stream_t stream);
int b2p_layerdrop_route(const float* dout, float* d_keep, float* d_skip, int64_t n, float p,
                        uint64_t seed, b2p_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* B2P_HIP_H */
