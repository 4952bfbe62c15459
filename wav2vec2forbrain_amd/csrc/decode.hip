// On-device greedy CTC decode + word error rate of a training batch: replaces the
// per-step host round trip of the reference's train evaluator (src/train/evaluator.py:69-129:
// logits.argmax(-1).cpu() -> tokenizer.batch_decode(group_tokens=True) -> cut after "</s>" ->
// torcheval WordErrorRate against batch_decode(target, group_tokens=False)).
//
// Token semantics restated from the wav2vec2 CTC tokenizer (transformers Wav2Vec2CTCTokenizer,
// convert_tokens_to_string): predictions group repeated ids, then drop the pad/blank id; targets
// only drop pads; the word-delimiter id separates words ("|" -> " ", and WER splits on
// whitespace, so empty words vanish); the prediction is cut after its first EOS id. Words are
// compared by a 64-bit hash of their id sequence (every vocab entry is one character or one
// special token, so equal id sequences <=> equal strings).
//
// One wave per sample: lanes take the frame argmaxes (first maximum, as torch.argmax), lane 0
// collapses, hashes the words and runs the word-level Levenshtein DP.
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {

constexpr int DEC_TMAX = 1024;
constexpr int DEC_WMAX = 512;

__device__ __forceinline__ uint64_t word_mix(uint64_t h, int id) {
  return (h ^ (uint64_t)(id + 1)) * 0x100000001B3ull;   // FNV-1a over the word's ids
}

__global__ void __launch_bounds__(64) ctc_greedy_wer_k(const float* __restrict__ logits, int T, int C,
                                                       const int64_t* __restrict__ target, int S, int blank,
                                                       int eos, int delim, int32_t* __restrict__ out_tok,
                                                       int32_t* __restrict__ out_ntok, int32_t* __restrict__ errs,
                                                       int32_t* __restrict__ nwords) {
  __shared__ int ids[DEC_TMAX];
  __shared__ uint64_t pw[DEC_WMAX], lw[DEC_WMAX];
  __shared__ int row[DEC_WMAX + 1];
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* lg = logits + (int64_t)b * T * C;
  for (int t = lane; t < T; t += 64) {
    const float* r = lg + (int64_t)t * C;
    float best = r[0];
    int bi = 0;
    for (int c = 1; c < C; ++c) {
      const float v = r[c];
      if (v > best || (v != v && best == best)) { best = v; bi = c; }   // NaN wins, like torch.argmax
    }
    ids[t] = bi;
  }
  __syncthreads();
  if (lane != 0) return;
  // prediction: group repeats, drop blanks, cut after the first EOS; words at delimiters
  int np = 0, nt = 0, last = -1, wlen = 0;
  uint64_t h = 0xCBF29CE484222325ull;
  int32_t* ot = out_tok + (int64_t)b * T;
  for (int t = 0; t < T; ++t) {
    const int id = ids[t];
    if (id == last) continue;
    last = id;
    if (id == blank) continue;
    ot[nt++] = id;
    if (id == delim) {
      if (wlen > 0 && np < DEC_WMAX) pw[np++] = h;
      h = 0xCBF29CE484222325ull;
      wlen = 0;
    } else {
      h = word_mix(h, id);
      ++wlen;
    }
    if (id == eos) break;
  }
  if (wlen > 0 && np < DEC_WMAX) pw[np++] = h;
  out_ntok[b] = nt;
  // target: drop pads, words at delimiters
  int nl = 0;
  wlen = 0;
  h = 0xCBF29CE484222325ull;
  const int64_t* tg = target + (int64_t)b * S;
  for (int s = 0; s < S; ++s) {
    const int id = (int)tg[s];
    if (id == blank) continue;
    if (id == delim) {
      if (wlen > 0 && nl < DEC_WMAX) lw[nl++] = h;
      h = 0xCBF29CE484222325ull;
      wlen = 0;
    } else {
      h = word_mix(h, id);
      ++wlen;
    }
  }
  if (wlen > 0 && nl < DEC_WMAX) lw[nl++] = h;
  // word-level Levenshtein distance (one DP row in LDS)
  for (int j = 0; j <= nl; ++j) row[j] = j;
  for (int i = 1; i <= np; ++i) {
    int diag = row[0];
    row[0] = i;
    for (int j = 1; j <= nl; ++j) {
      const int up = row[j];
      const int sub = diag + (pw[i - 1] != lw[j - 1] ? 1 : 0);
      int v = up + 1 < row[j - 1] + 1 ? up + 1 : row[j - 1] + 1;
      row[j] = v < sub ? v : sub;
      diag = up;
    }
  }
  errs[b] = row[nl];
  nwords[b] = nl;
}

// ---- character error rate (reference EvaluatorWithW2vLMDecoder.calculate_char_error_rate,
// src/train/evaluator.py:212-214,231-242: edit_distance.SequenceMatcher(a=target, b=prediction)
// .distance() summed over the batch, / summed target lengths). The strings are rebuilt from the
// tokens exactly as Wav2Vec2CTCTokenizer renders them: every token expands to its characters
// (tok_chars[id][0..tok_len[id]), e.g. "</s>" is 4 characters), the word delimiter renders as ' ',
// the whole string is stripped of surrounding spaces and the prediction is cut after its first
// "</s>". The Levenshtein DP runs one anti-diagonal per step across the 64 lanes of the wave.
constexpr int CER_CMAX = 2048;

__global__ void __launch_bounds__(64) ctc_greedy_cer_k(const float* __restrict__ logits, int T, int C,
                                                       const int64_t* __restrict__ target, int S, int blank,
                                                       int eos, int delim, const uint8_t* __restrict__ tok_chars,
                                                       const int32_t* __restrict__ tok_len,
                                                       int32_t* __restrict__ char_errs, int32_t* __restrict__ nchars) {
  __shared__ int ids[DEC_TMAX];
  __shared__ uint8_t pc[CER_CMAX], tc[CER_CMAX];
  __shared__ int diag[3][CER_CMAX + 1];
  __shared__ int lens[2];
  const int b = blockIdx.x, lane = threadIdx.x;
  const float* lg = logits + (int64_t)b * T * C;
  for (int t = lane; t < T; t += 64) {
    const float* r = lg + (int64_t)t * C;
    float best = r[0];
    int bi = 0;
    for (int c = 1; c < C; ++c) {
      const float v = r[c];
      if (v > best || (v != v && best == best)) { best = v; bi = c; }
    }
    ids[t] = bi;
  }
  __syncthreads();
  if (lane == 0) {
    bool over = false;
    // prediction: group repeats, drop blanks, render, strip leading spaces, cut after the first EOS
    // (or strip trailing spaces when there is none)
    int np = 0, last = -1;
    bool cut = false;
    for (int t = 0; t < T && !cut; ++t) {
      const int id = ids[t];
      if (id == last) continue;
      last = id;
      if (id == blank) continue;
      const int n = id == delim ? 1 : tok_len[id];
      for (int k = 0; k < n; ++k) {
        const uint8_t ch = id == delim ? (uint8_t)' ' : tok_chars[id * 8 + k];
        if (np == 0 && ch == ' ') continue;
        if (np < CER_CMAX) pc[np++] = ch; else over = true;
      }
      cut = id == eos;
    }
    if (!cut) while (np > 0 && pc[np - 1] == ' ') --np;
    // target: drop pads (no grouping), render, strip both ends
    int nt = 0;
    for (int s = 0; s < S; ++s) {
      const int id = (int)target[(int64_t)b * S + s];
      if (id == blank || id < 0 || id >= C) continue;
      const int n = id == delim ? 1 : tok_len[id];
      for (int k = 0; k < n; ++k) {
        const uint8_t ch = id == delim ? (uint8_t)' ' : tok_chars[id * 8 + k];
        if (nt == 0 && ch == ' ') continue;
        if (nt < CER_CMAX) tc[nt++] = ch; else over = true;
      }
    }
    while (nt > 0 && tc[nt - 1] == ' ') --nt;
    lens[0] = over ? -1 : nt;
    lens[1] = np;
  }
  __syncthreads();
  const int L = lens[0], P = lens[1];
  if (L < 0) {   // longer than the LDS images: reported, not guessed
    if (lane == 0) { char_errs[b] = -1; nchars[b] = 0; }
    return;
  }
  // D[i][j] = distance(target[:i], pred[:j]); anti-diagonal k = i + j lives in diag[k % 3][i]
  for (int k = 0; k <= L + P; ++k) {
    int* d0 = diag[k % 3];
    const int* d1 = diag[(k + 2) % 3];
    const int* d2 = diag[(k + 1) % 3];
    const int lo = k - P > 0 ? k - P : 0, hi = k < L ? k : L;
    for (int i = lo + lane; i <= hi; i += 64) {
      const int j = k - i;
      int v;
      if (i == 0) v = j;
      else if (j == 0) v = i;
      else {
        const int sub = d2[i - 1] + (tc[i - 1] != pc[j - 1] ? 1 : 0);
        const int del = d1[i - 1] + 1;
        const int ins = d1[i] + 1;
        v = sub < del ? sub : del;
        v = v < ins ? v : ins;
      }
      d0[i] = v;
    }
    __syncthreads();
  }
  if (lane == 0) {
    char_errs[b] = diag[(L + P) % 3][L];
    nchars[b] = L;
  }
}

}  // namespace

extern "C" int b2p_ctc_greedy_cer(const float* logits, int64_t B, int64_t T, int64_t C, const int64_t* target,
                                  int64_t S, int blank, int eos, int delim, const uint8_t* tok_chars,
                                  const int32_t* tok_len, int32_t* char_errs, int32_t* nchars, b2p_stream_t stream) {
  B2P_CHECK_ARG(logits && target && tok_chars && tok_len && char_errs && nchars, "ctc_greedy_cer: NULL pointer");
  B2P_CHECK_ARG(T >= 1 && T <= DEC_TMAX && C >= 1 && S >= 0, "ctc_greedy_cer: T must be in [1, %d]", DEC_TMAX);
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ctc_greedy_cer_k, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream, logits, (int)T, (int)C,
                     target, (int)S, blank, eos, delim, tok_chars, tok_len, char_errs, nchars);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_ctc_greedy_wer(const float* logits, int64_t B, int64_t T, int64_t C, const int64_t* target,
                                  int64_t S, int blank, int eos, int delim, int32_t* out_tokens, int32_t* out_ntok,
                                  int32_t* errs, int32_t* nwords, b2p_stream_t stream) {
  B2P_CHECK_ARG(logits && target && out_tokens && out_ntok && errs && nwords, "ctc_greedy_wer: NULL pointer");
  B2P_CHECK_ARG(T >= 1 && T <= DEC_TMAX && C >= 1 && S >= 0, "ctc_greedy_wer: T must be in [1, %d]", DEC_TMAX);
  if (B <= 0) return 0;
  hipLaunchKernelGGL(ctc_greedy_wer_k, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream, logits, (int)T, (int)C,
                     target, (int)S, blank, eos, delim, out_tokens, out_ntok, errs, nwords);
  B2P_CHECK_LAUNCH();
  return 0;
}
