// Fused bf16-MFMA self-attention (forward + backward) for the w2v / Conformer encoder layers:
// softmax(Q K^T * scale) -> dropout -> @ V, no mask (reference: HF Wav2Vec2Attention / eager
// attention, TF w2v:438-463,529-545; Conformer TF conf:458-470). bf16 precision mode only.
//
// T' <= 512 and head size 64 (TM = 256: T' = 249 frames at the 1024-bin windows; TM = 512: windows up
// to 2,080 bins), so one (batch, head)'s whole K and V fit in 64 / 128 KB of LDS: no online softmax is
// needed. Scores never touch HBM (the unfused
// path writes and re-reads a (B, heads, T', T') fp32 tensor ~6 times per layer).
//   fwd   (b, h, 128-query block): S^T = K Q^T (keys in registers, query on the lane), in-register
//         softmax (2 cross-lane shuffles per reduction), O^T = V^T P^T with P^T taken straight
//         from the accumulators as the B operand and V^T read by ds_read_b64_tr_b16.
//         Saves lse2[b][h][q] = max + log2(sum) in the log2 domain.
//   dQ    (b, h, 128-query block, launched first): S^T, dP^T recomputed from lse2 (no stored
//         probabilities); delta = sum_key P_d dP_d; dQ^T += K^T dS^T.
//   dK/dV (b, h, 128-key block): S, dP = dO V^T with the key on the lane; dV^T += dO^T P_d and
//         dK^T += Q^T dS with the dQ pass's delta.
// Dropout: keep(b, h, q, key) = b2p_keep(seed, ((b*nh + h)*T + q)*TP + key), TP = T rounded up to
// even (a hash serves an aligned pair of keys) — the same mask the unfused softmax kernel draws
// (b2p_softmax_fwd), so both paths agree element for element.
#include "common.h"
#include <type_traits>
#include <stdlib.h>
#include "../../include/b2p_hip.h"

namespace {
constexpr int DH = 64;     // head size
constexpr int TMAX = 256;  // sequence-length class of the stored keep mask (keys / queries <= 256)
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr float LOG2E = 1.4426950408889634f;

// [256 rows][64 bf16] LDS image, 16-byte chunks XOR-swizzled by row (conflict-light row reads)
__device__ __forceinline__ int img_off(int row, int col) {
  return row * 128 + ((((col >> 3) ^ row) & 7) << 4) + ((col & 7) << 1);
}
// A/B fragment of v_mfma_f32_16x16x32_bf16 read along a row: 8 bf16 at (row, col..col+7)
__device__ __forceinline__ bf16x8 row_frag(const char* img, int row, int col) {
  return *reinterpret_cast<const bf16x8*>(img + img_off(row, col));
}
// transposed fragment: element q (0..3) = img[r0 + q][c0 + lane%16] via ds_read_b64_tr_b16, for
// the two 4-row blocks r0 and r1 (elements 0..3 and 4..7)
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int r0, int r1, int c0, int li) {
  const int q = li >> 2, p = li & 3;
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + img_off(r0 + q, c0 + 4 * p)));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + img_off(r1 + q, c0 + 4 * p)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ bf16x8 pack_acc(const f32x4& a, const f32x4& b) {
  bf16x8 r = {(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)a[3],
              (__bf16)b[0], (__bf16)b[1], (__bf16)b[2], (__bf16)b[3]};
  return r;
}
__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// H: the 16-bit containers hold fp16 bits (v_mfma_f32_16x16x32_f16), else bf16
typedef _Float16 f16x8a __attribute__((ext_vector_type(8)));
template <bool H>
__device__ __forceinline__ f32x4 mfma_t(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8a, a), __builtin_bit_cast(f16x8a, b), c, 0,
                                                  0, 0);
  else
    return mfma(a, b, c);
}
template <bool H>
__device__ __forceinline__ bf16x8 pack_acc_t(const f32x4& a, const f32x4& b) {
  if constexpr (H) {
    f16x8a r = {(_Float16)a[0], (_Float16)a[1], (_Float16)a[2], (_Float16)a[3],
                (_Float16)b[0], (_Float16)b[1], (_Float16)b[2], (_Float16)b[3]};
    return __builtin_bit_cast(bf16x8, r);
  } else {
    return pack_acc(a, b);
  }
}
__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

// Load rows [0, TM) of a head slice (64 bf16 at column `col` of a row-major [B*T][ld] bf16
// matrix) into an LDS image; rows >= T are zero. 256 threads, 8 chunks of 16 B each.
template <int TM>
__device__ __forceinline__ void load_image(char* img, const uint16_t* base, int64_t row0, int T, int64_t ld, int col,
                                           int tid) {
#pragma unroll
  for (int k = 0; k < TM / 32; ++k) {
    const int idx = tid + 256 * k;
    const int r = idx >> 3, c = idx & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < T) v = *reinterpret_cast<const uint4*>(base + (row0 + r) * ld + col + 8 * c);
    *reinterpret_cast<uint4*>(img + r * 128 + (((c ^ r) & 7) << 4)) = v;
  }
}
__device__ __forceinline__ bf16x8 gload8(const uint16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
// 8 fp16 values (bits in a bf16x8 container) -> bf16 (the backward's products with bf16 gradients)
__device__ __forceinline__ bf16x8 h2b8(const bf16x8& x) {
  const f16x8a h = __builtin_bit_cast(f16x8a, x);
  bf16x8 r = {(__bf16)(float)h[0], (__bf16)(float)h[1], (__bf16)(float)h[2], (__bf16)(float)h[3],
              (__bf16)(float)h[4], (__bf16)(float)h[5], (__bf16)(float)h[6], (__bf16)(float)h[7]};
  return r;
}
template <bool H>
__device__ __forceinline__ bf16x8 to_b16(const bf16x8& x) {
  if constexpr (H) return h2b8(x);
  else return x;
}
// load_image with each 16-B chunk converted fp16 -> bf16 on the way (H), else a plain copy
template <bool H, int TM>
__device__ __forceinline__ void load_image_b16(char* img, const uint16_t* base, int64_t row0, int T, int64_t ld,
                                               int col, int tid) {
#pragma unroll
  for (int k = 0; k < TM / 32; ++k) {
    const int idx = tid + 256 * k;
    const int r = idx >> 3, c = idx & 7;
    bf16x8 v = bf16x8{};
    if (r < T) v = to_b16<H>(gload8(base + (row0 + r) * ld + col + 8 * c));
    *reinterpret_cast<bf16x8*>(img + r * 128 + (((c ^ r) & 7) << 4)) = v;
  }
}
__device__ __forceinline__ void store_out(float* o32, uint16_t* o16, int64_t off, const f32x4& v, float s) {
  const float4 f = make_float4(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
  if (o32) *reinterpret_cast<float4*>(o32 + off) = f;
  if (o16) *reinterpret_cast<uint2*>(o16 + off) = b2p_pack_bf16x4(f);
}

struct DropCfg {
  uint64_t seed;
  uint32_t thr;
  float scale;                // 1 / (1 - p)
  const uint64_t* epoch;      // graph-replay seed offset (b2p_seed_eff), NULL in eager launches
  const int32_t* gate;        // LayerDrop gate (b2p_gate): closed -> fwd does nothing, bwd writes zeros
};

// closed-gate backward: zero this block's 64 rows x 64 columns of dqkv at column col (fp32 and/or bf16)
__device__ __forceinline__ void zero_block(float* dqkv, uint16_t* dqkv16, int64_t row0, int r0, int T, int64_t ld,
                                           int64_t col, int tid) {
  for (int i = tid; i < 64 * 16; i += 256) {
    const int r = r0 + (i >> 4);
    if (r >= T) continue;
    const int64_t o = (row0 + r) * ld + col + 4 * (i & 15);
    if (dqkv) *reinterpret_cast<float4*>(dqkv + o) = make_float4(0.f, 0.f, 0.f, 0.f);
    if (dqkv16) *reinterpret_cast<uint2*>(dqkv16 + o) = make_uint2(0u, 0u);
  }
}
template <bool DROP>
__device__ __forceinline__ float keep_scale(const DropCfg& dc, uint64_t idx) {
  if (!DROP) return 1.f;
  return b2p_keep(dc.seed, idx, dc.thr) ? dc.scale : 0.f;
}

// ------------------------------------------------------------------------------------------ forward
// qkv16 [B*T][3*D] bf16 (q | k | v, head-major inside each); O16 [B*T][D] bf16; lse2 [B][nh][T]
// H (b2p_attn16_fwd_f16): qkv16 and O16 hold fp16 and both products run on fp16 MFMA (P in fp16: 11
// significant bits instead of 8); Ob16, when given, receives a bf16 copy of O (the backward's
// weight-gradient operand)
// One workgroup per (batch, head, 128-query half): 4 waves stage K and V once (64 KB of LDS) and then
// each wave runs query tiles w and w + 4 of its half (16 queries each). K/V cross L2 -> LDS once per
// 128 queries (half the traffic of 64-query blocks), and 2 x B x heads workgroups (768 at the base
// workload) spread evenly over 256 CUs at two resident workgroups per CU.
// Dropout keep bits come two per hash (b2p_hash of idx >> 1, 16-bit halves) with the row stride TP
// = T rounded up to even, so a lane's 4 consecutive keys need exactly 2 hashes.
constexpr int FWD_NT = 256;
// Stored keep mask: 32 bytes per query row, byte 8*g + c (g = (key >> 2) & 3, c = key >> 5) holds keys
// 32c + 4g + i (bit i) and 32c + 16 + 4g + i (bit 4 + i): each forward lane writes its own 8 bytes.
// Within 32-bit word (key >> 5) / 4 + 2g of the row: bit position of key
__device__ __forceinline__ int mask_shift(int key) { return 8 * ((key >> 5) & 3) + 4 * ((key >> 4) & 1) + (key & 3); }
#ifndef B2P_ATTN_QB
#define B2P_ATTN_QB 128
#endif
constexpr int FWD_QB = B2P_ATTN_QB;   // queries per workgroup (forward and dQ)
// the 4 keep bits of keys key0 .. key0+3 (key0 % 4 == 0) of mask row `row` (32-bit element index:
// b2p_hash with idx >> 32 == 0, checked on the host)
__device__ __forceinline__ uint32_t keep4_bits(uint32_t key_lo, uint32_t k32, uint32_t thr16) {
#ifdef B2P_HASH_1R
  const uint32_t h0 = b2p_mix32((key_lo >> 1) ^ k32);
  const uint32_t h1 = b2p_mix32(((key_lo >> 1) + 1) ^ k32);
#else
  const uint32_t h0 = b2p_mix32(b2p_mix32((key_lo >> 1) ^ k32) + k32);
  const uint32_t h1 = b2p_mix32(b2p_mix32(((key_lo >> 1) + 1) ^ k32) + k32);
#endif
  // (v - thr16) >> 31 = 1 exactly when v < thr16 (v, thr16 <= 2^16): the drop bits by arithmetic (compares
  // would each tie up an SGPR pair across the unrolled loop)
  const uint32_t d = (((h0 & 0xFFFFu) - thr16) >> 31) | ((((h0 >> 16) - thr16) >> 31) << 1) |
                     ((((h1 & 0xFFFFu) - thr16) >> 31) << 2) | ((((h1 >> 16) - thr16) >> 31) << 3);
  return d ^ 0xFu;
}

// T1: T > TM - 16, so keys >= T lie in the last key tile only: its score accumulator starts from a bias
// (0 for keys < T, -inf beyond) computed once, and no per-element masking runs in the loop (the masked
// form's uniform per-tile branches made the unrolled loop spill ~230 SGPRs into VGPR lanes)
// DM 0: no dropout, 1: hash the keep mask, 2: also store the keep bits for the backward, 3: read the keep
// bits from maskw (drawn ahead by attn_keep_k, the layout DM 2 stores)
template <int DM, bool H, int TM, bool T1 = false>
__global__ void __launch_bounds__(FWD_NT) attn16_fwd_k(const uint16_t* __restrict__ qkv, uint16_t* __restrict__ O16,
                                                       uint16_t* __restrict__ Ob16, float* __restrict__ lse2, int T,
                                                       int nh, float scale, DropCfg dc, uint32_t* __restrict__ maskw) {
  static_assert(TM == TMAX || DM < 2, "the stored keep mask covers T <= 256");
  constexpr int NKT = TM / 16;   // key tiles
  constexpr bool DROP = DM != 0;
  if (b2p_gated_off(dc.gate)) return;   // LayerDrop: this replay skips the layer (outputs unused)
  dc.seed = b2p_seed_eff(dc.seed, dc.epoch);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqh = (T + FWD_QB - 1) / FWD_QB;
  const int bh = blockIdx.x / nqh, qh = blockIdx.x - bh * nqh;
  const int b = bh / nh, h = bh - b * nh;
  const int D = nh * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, g = l >> 4;
  const int64_t row0 = (int64_t)b * T;
  const int TP = T + (T & 1);
  // this wave's first query tile: its Q fragments are in flight while K / V are staged
  bf16x8 qf[2];
  const int qt0 = qh * (FWD_QB / 16) + w;
  {
    const int q = qt0 * 16 + lr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[ks] = q < T ? gload8(qkv + (row0 + q) * ld + h * DH + 32 * ks + 8 * g) : bf16x8{};
  }
  load_image<TM>(smem, qkv, row0, T, ld, D + h * DH, tid);
  load_image<TM>(smem + TM * 128, qkv, row0, T, ld, 2 * D + h * DH, tid);
  __syncthreads();
  const float c2 = scale * LOG2E;
  const uint32_t k32 = (uint32_t)dc.seed ^ b2p_mix32((uint32_t)(dc.seed >> 32) + 0x9E3779B9u);   // b2p_hash key
  const uint32_t thr16 = b2p_thr16(dc.thr);
  f32x4 tail0 = f32x4{0.f, 0.f, 0.f, 0.f};   // T1: the last key tile's initial scores (0 / -inf)
  if constexpr (T1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) tail0[i] = (NKT - 1) * 16 + 4 * g + i < T ? 0.f : -INFINITY;
  }
  for (int qt = qt0; qt < qt0 + FWD_QB / 16 && qt * 16 < T; qt += 4) {
    // opaque per-iteration image bases: keeps the compiler from hoisting the ~100 per-lane LDS
    // fragment addresses of the unrolled body out of the loop (they would not fit beside s[16])
    uint32_t obase = 0;
    asm volatile("" : "+v"(obase));
    const char* Kimg = smem + obase;
    const char* Vimg = smem + TM * 128 + obase;
    const int q = qt * 16 + lr;
    const bool qok = q < T;
    uint32_t mbits[2] = {0u, 0u};   // this lane's keep bits: byte c = keys 32c + 4g + i (bit i), +16 (bit 4 + i)
    if constexpr (DM == 3) {        // issued first: the load hides under the S MFMAs
      if (qok) {
        const uint2 mw = *reinterpret_cast<const uint2*>(maskw + (((int64_t)b * nh + h) * T + q) * 8 + 2 * g);
        mbits[0] = mw.x;
        mbits[1] = mw.y;
      }
    }
    if (qt != qt0) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) qf[ks] = qok ? gload8(qkv + (row0 + q) * ld + h * DH + 32 * ks + 8 * g) : bf16x8{};
    }
    // S^T: tile kt = keys kt*16 + 4g + i (registers) x query q (lane)
    f32x4 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = (T1 && kt == NKT - 1) ? tail0 : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) s[kt] = mfma_t<H>(row_frag(Kimg, kt * 16 + lr, 32 * ks + 8 * g), qf[ks], s[kt]);
    }
    // row max of the raw scores (scale > 0 commutes with max); keys >= T are masked only in the tiles
    // that hold them (wave-uniform test; T1: already -inf from the accumulator's start), the scale is
    // folded into the exponent's FMA
    float m = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (T1 || kt * 16 + 16 <= T) {
#pragma unroll
        for (int i = 0; i < 4; ++i) m = fmaxf(m, s[kt][i]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = kt * 16 + 4 * g + i < T ? s[kt][i] : -INFINITY;
          s[kt][i] = v;
          m = fmaxf(m, v);
        }
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    const float mc = m * c2;
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = exp2_fast(fmaf(s[kt][i], c2, -mc));
        s[kt][i] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    const float inv = 1.f / sum;
    const float inv_s = DROP ? inv * dc.scale : inv;   // keys >= T already hold exp2(-inf) = 0
    const uint32_t rowlo = (uint32_t)((((uint32_t)b * (uint32_t)nh + (uint32_t)h) * (uint32_t)T + (uint32_t)(qok ? q : 0)) *
                                      (uint32_t)TP);
    // O^T (d x q) = V^T (d x keys) . P_d^T (keys x q), 32 keys per k-step
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NKT / 2; ++c) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int key0 = (2 * c + half) * 16 + 4 * g;
        const uint32_t kb = DM == 3 ? (mbits[c >> 2] >> (8 * (c & 3) + 4 * half)) & 0xFu
                            : DROP  ? keep4_bits(rowlo + (uint32_t)key0, k32, thr16)
                                    : 0xFu;
        if (DM == 2) mbits[c >> 2] |= kb << (8 * (c & 3) + 4 * half);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = s[2 * c + half][i] * inv_s;
          if constexpr (DROP) {   // keep bit i as an all-ones / zero mask: bit arithmetic, no compare masks
            const uint32_t km = (uint32_t)((int32_t)(kb << (31 - i)) >> 31);
            s[2 * c + half][i] = __uint_as_float(__float_as_uint(pv) & km);
          } else {
            s[2 * c + half][i] = pv;
          }
        }
      }
      const bf16x8 bp = pack_acc_t<H>(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        o[dt] = mfma_t<H>(tr_frag(Vimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr), bp, o[dt]);
    }
    // the keep bits for the backward kernels, each lane's own 8 bytes: mask row (32 bytes per query)
    // = [lane group g][chunk c] bytes (mask_bit() below)
    if (DM == 2 && qok)
      *reinterpret_cast<uint2*>(maskw + (((int64_t)b * nh + h) * T + q) * 8 + 2 * g) = make_uint2(mbits[0], mbits[1]);
    const int64_t orow = (row0 + q) * D + h * DH;
    if (qok) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int64_t off = orow + dt * 16 + 4 * g;
        if constexpr (H) {
          *reinterpret_cast<uint2*>(O16 + off) = b2p_pack16x4(make_float4(o[dt][0], o[dt][1], o[dt][2], o[dt][3]), true);
          if (Ob16) store_out(nullptr, Ob16, off, o[dt], 1.f);
        } else {
          store_out(nullptr, O16, off, o[dt], 1.f);
        }
      }
    }
    if (qok && g == 0) lse2[((int64_t)b * nh + h) * T + q] = mc + __log2f(sum);
  }
}

// Dropout keep bits of several layers' attention in one launch (b2p_attn16_keep_masks): for each layer's
// seed, word for word the mask a DM 2 forward stores, so that layer's forward reads its bits (DM 3)
// instead of hashing them in its VALU-bound softmax loop, and the backward reads them as before. The
// model forward issues it on a side stream at its start (functional.attn_keep_plan). One thread per (layer, batch x head x query row, lane group g): the 16 keep4_bits
// of the 8 bytes forward lane (g, query) writes.
constexpr int KEEP_LAYERS = 32;   // layers per launch (seeds by value)
constexpr int KEEP_LDS = 24 * 1024;
struct KeepSeeds {
  uint64_t seed[KEEP_LAYERS];
};
__global__ void __launch_bounds__(256) attn_keep_k(uint32_t* __restrict__ mask, KeepSeeds ks,
                                                   const uint64_t* __restrict__ epoch, int64_t rows, int T,
                                                   uint32_t thr, int nl) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = rows * 4;
  if (i >= per * nl) return;
  const int layer = (int)(i / per);
  const int64_t r = i - layer * per;
  const int64_t row = r >> 2;   // (b * nh + h) * T + q
  const int g = (int)(r & 3);
  const uint64_t seed = b2p_seed_eff(ks.seed[layer], epoch);
  const uint32_t k32 = (uint32_t)seed ^ b2p_mix32((uint32_t)(seed >> 32) + 0x9E3779B9u);
  const uint32_t thr16 = b2p_thr16(thr);
  const uint32_t rowlo = (uint32_t)row * (uint32_t)(T + (T & 1));
  uint32_t mb[2] = {0u, 0u};
#pragma unroll
  for (int c = 0; c < TMAX / 32; ++c)
#pragma unroll
    for (int half = 0; half < 2; ++half)
      mb[c >> 2] |= keep4_bits(rowlo + (uint32_t)((2 * c + half) * 16 + 4 * g), k32, thr16) << (8 * (c & 3) + 4 * half);
  *reinterpret_cast<uint2*>(mask + (int64_t)layer * rows * 8 + row * 8 + 2 * g) = make_uint2(mb[0], mb[1]);
}

// ------------------------------------------------------------------------------------ backward dK dV
// dO16 [B*T][D] bf16; delta [B][nh][T] from the dQ kernel; writes dK, dV into dqkv (fp32 and/or
// bf16) columns [D + h*64, ...) and [2D + h*64, ...). One workgroup per (batch, head, 128 keys): Q and
// dO are staged once for 128 keys (4 waves x key tiles w and w + 4).
constexpr int BWD_KB = 128;
template <int DM, bool H, int TM>   // DM 0: no dropout, 1: hash the keep mask, 2: keep bits in memory; H: fp16 qkv
__global__ void __launch_bounds__(256) attn16_bwd_dkv_k(const uint16_t* __restrict__ qkv, const float* __restrict__ delta,
                                                        const uint16_t* __restrict__ dO16, const float* __restrict__ lse2,
                                                        float* __restrict__ dqkv, uint16_t* __restrict__ dqkv16, int T,
                                                        int nh, float scale, DropCfg dc,
                                                        const uint32_t* __restrict__ maskw) {
  static_assert(TM == TMAX || DM != 2, "the stored keep mask covers T <= 256");
  constexpr bool DROP = DM != 0;
  dc.seed = b2p_seed_eff(dc.seed, dc.epoch);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* lse_s = reinterpret_cast<float*>(smem + 2 * TM * 128);
  float* del_s = lse_s + TM;
  uint32_t* msk_s = reinterpret_cast<uint32_t*>(del_s + TM);   // [q][4]: this block's 128 keys' bits (TM 256)
  const int nkb = (T + BWD_KB - 1) / BWD_KB;
  const int bhi = blockIdx.x / nkb, kb = blockIdx.x - bhi * nkb;
  const int b = bhi / nh, h = bhi - b * nh;
  const int D = nh * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, g = l >> 4;
  const int64_t row0 = (int64_t)b * T;
  if (b2p_gated_off(dc.gate)) {   // LayerDrop: zero dK, dV (the bias reduction reads them)
    for (int half = 0; half < 2; ++half) {
      zero_block(dqkv, dqkv16, row0, kb * BWD_KB + 64 * half, T, ld, D + h * DH, tid);
      zero_block(dqkv, dqkv16, row0, kb * BWD_KB + 64 * half, T, ld, 2 * D + h * DH, tid);
    }
    return;
  }
  load_image<TM>(smem, qkv, row0, T, ld, h * DH, tid);
  load_image<TM>(smem + TM * 128, dO16, row0, T, D, h * DH, tid);
  for (int qq = tid; qq < TM; qq += 256) {   // one thread per query row: lse2 and delta (from the dQ pass)
    const int64_t o = ((int64_t)b * nh + h) * T + qq;
    del_s[qq] = qq < T ? delta[o] : 0.f;
    lse_s[qq] = qq < T ? lse2[o] : 0.f;
    if (DM == 2) {   // the keep bits of keys 128kb .. 128kb+127 for every query row: word 2g + kb, g = 0..3
#pragma unroll
      for (int j = 0; j < 4; ++j) msk_s[4 * qq + j] = qq < T ? maskw[o * 8 + 2 * j + kb] : 0u;
    }
  }
  __syncthreads();
  const float c2 = scale * LOG2E;
  const uint64_t bh = (uint64_t)b * nh + h;
  const int TP = T + (T & 1);
  const int kt0 = kb * (BWD_KB / 16) + w;
  for (int kt = kt0; kt < kt0 + BWD_KB / 16 && kt * 16 < T; kt += 4) {
    uint32_t obase = 0;   // opaque image bases: no hoisting of the unrolled body's LDS addresses
    asm volatile("" : "+v"(obase));
    const char* Qimg = smem + obase;
    const char* dOimg = smem + TM * 128 + obase;
    const int key = kt * 16 + lr;
    const bool kok = key < T;
    const int kw = (key >> 2) & 3;                 // this key's word among the block's 4 (its lane group)
    const int ksh = mask_shift(key);
    bf16x8 kf[2], vf[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = vf[ks] = bf16x8{};
      if (kok) {
        kf[ks] = gload8(qkv + (row0 + key) * ld + D + h * DH + 32 * ks + 8 * g);
        vf[ks] = to_b16<H>(gload8(qkv + (row0 + key) * ld + 2 * D + h * DH + 32 * ks + 8 * g));
      }
    }
    f32x4 dv[4], dk[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dv[dt] = dk[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nchunk = (T + 31) >> 5;
    for (int c = 0; c < nchunk; ++c) {
      f32x4 pd[2], ds[2];
      uint32_t mw[2][4];   // keep-bit words (from the forward, staged in LDS) of this chunk's queries
      if (DM == 2) {
#pragma unroll
        for (int half = 0; half < 2; ++half)
#pragma unroll
          for (int i = 0; i < 4; ++i) mw[half][i] = msk_s[4 * ((2 * c + half) * 16 + 4 * g + i) + kw];
      }
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int qt = 2 * c + half;
        f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sv = mfma_t<H>(row_frag(Qimg, qt * 16 + lr, 32 * ks + 8 * g), kf[ks], sv);
          dp = mfma(row_frag(dOimg, qt * 16 + lr, 32 * ks + 8 * g), vf[ks], dp);
        }
        // rows q = qt*16 + 4g + i, column key
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = qt * 16 + 4 * g + i;
          const bool ok = kok && qq < T;
          const float p = ok ? exp2_fast(fmaf(sv[i], c2, -lse_s[qq])) : 0.f;
          const float ksc = !ok ? 0.f
                            : (DM == 2) ? (((mw[half][i] >> ksh) & 1u) ? dc.scale : 0.f)
                                              : keep_scale<DROP>(dc, (bh * T + qq) * (uint64_t)TP + key);
          pd[half][i] = p * ksc;
          ds[half][i] = p * (dp[i] * ksc - del_s[qq]);
        }
      }
      const bf16x8 bp = pack_acc(pd[0], pd[1]), bs = pack_acc(ds[0], ds[1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma(tr_frag(dOimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr), bp, dv[dt]);
        dk[dt] = mfma(to_b16<H>(tr_frag(Qimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr)), bs, dk[dt]);
      }
    }
    if (kok) {
      const int64_t r = (row0 + key) * ld + h * DH;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store_out(dqkv, dqkv16, r + D + dt * 16 + 4 * g, dk[dt], scale);
        store_out(dqkv, dqkv16, r + 2 * D + dt * 16 + 4 * g, dv[dt], 1.f);
      }
    }
  }
}

// Paired form: each wave runs its two key tiles (w and w + 4 of the block) in ONE pass over the queries,
// so every Q / dO fragment read from LDS, every fp16 -> bf16 conversion of the Q^T operand, every lse2 /
// delta / keep-word read serves both tiles (the per-tile form repeats them per tile: the conversions
// alone were ~50 VALU per 32-query chunk and tile). Keep words are staged [word][query] (rows padded by
// 8 words: the 4 words a 32-lane half reads land on distinct banks) so a lane's 4 consecutive queries
// are one 16-byte read; validity and keep are all-ones / zero bit masks. Accumulation order per tile
// is the per-tile kernel's, so both forms write bitwise-equal dK / dV.
constexpr int MSK_LD = TMAX + 8;
template <int DM, bool H, int TM>
__global__ void __launch_bounds__(256) attn16_bwd_dkv2_k(const uint16_t* __restrict__ qkv, const float* __restrict__ delta,
                                                         const uint16_t* __restrict__ dO16, const float* __restrict__ lse2,
                                                         float* __restrict__ dqkv, uint16_t* __restrict__ dqkv16, int T,
                                                         int nh, float scale, DropCfg dc,
                                                         const uint32_t* __restrict__ maskw) {
  static_assert(TM == TMAX || DM != 2, "the stored keep mask covers T <= 256");
  constexpr bool DROP = DM != 0;
  dc.seed = b2p_seed_eff(dc.seed, dc.epoch);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* lse_s = reinterpret_cast<float*>(smem + 2 * TM * 128);
  float* del_s = lse_s + TM;
  uint32_t* msk_s = reinterpret_cast<uint32_t*>(del_s + TM);   // [word j][query], row stride MSK_LD (TM 256)
  const int nkb = (T + BWD_KB - 1) / BWD_KB;
  const int bhi = blockIdx.x / nkb, kb = blockIdx.x - bhi * nkb;
  const int b = bhi / nh, h = bhi - b * nh;
  const int D = nh * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, g = l >> 4;
  const int64_t row0 = (int64_t)b * T;
  if (b2p_gated_off(dc.gate)) {   // LayerDrop: zero dK, dV (the bias reduction reads them)
    for (int half = 0; half < 2; ++half) {
      zero_block(dqkv, dqkv16, row0, kb * BWD_KB + 64 * half, T, ld, D + h * DH, tid);
      zero_block(dqkv, dqkv16, row0, kb * BWD_KB + 64 * half, T, ld, 2 * D + h * DH, tid);
    }
    return;
  }
  load_image<TM>(smem, qkv, row0, T, ld, h * DH, tid);
  load_image<TM>(smem + TM * 128, dO16, row0, T, D, h * DH, tid);
  for (int qq = tid; qq < TM; qq += 256) {   // one thread per query row: lse2 and delta (from the dQ pass)
    const int64_t o = ((int64_t)b * nh + h) * T + qq;
    del_s[qq] = qq < T ? delta[o] : 0.f;
    lse_s[qq] = qq < T ? lse2[o] : 0.f;
    if (DM == 2) {   // the keep bits of keys 128kb .. 128kb+127 for every query row: word 2j + kb, j = 0..3
#pragma unroll
      for (int j = 0; j < 4; ++j) msk_s[j * MSK_LD + qq] = qq < T ? maskw[o * 8 + 2 * j + kb] : 0u;
    }
  }
  __syncthreads();
  const int kt0 = kb * (BWD_KB / 16) + w;
  if (kt0 * 16 >= T) return;   // both of this wave's key tiles lie beyond T (no barrier follows)
  const float c2 = scale * LOG2E;
  const uint64_t bh = (uint64_t)b * nh + h;
  const int TP = T + (T & 1);
  uint32_t obase = 0;   // opaque image bases: no hoisting of the unrolled body's LDS addresses
  asm volatile("" : "+v"(obase));
  const char* Qimg = smem + obase;
  const char* dOimg = smem + TM * 128 + obase;
  // tile t = key tile kt0 + 4t: keys key[t] = (kt0 + 4t) * 16 + lr on the lane
  int key[2];
  uint32_t kokm[2];
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    key[t] = (kt0 + 4 * t) * 16 + lr;
    const bool kok = key[t] < T;
    kokm[t] = 0u - (uint32_t)kok;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[t][ks] = vf[t][ks] = bf16x8{};
      if (kok) {
        kf[t][ks] = gload8(qkv + (row0 + key[t]) * ld + D + h * DH + 32 * ks + 8 * g);
        vf[t][ks] = to_b16<H>(gload8(qkv + (row0 + key[t]) * ld + 2 * D + h * DH + 32 * ks + 8 * g));
      }
    }
  }
  // keep bit of key[t] in its query's word (lr >> 2): mask_shift(key[0]) < 16, key[1] = key[0] + 64 -> +16
  const int kw = lr >> 2;
  const int ksh = mask_shift(key[0]);
  f32x4 dv[2][4], dk[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dv[t][dt] = dk[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nchunk = (T + 31) >> 5;
  for (int c = 0; c < nchunk; ++c) {
    f32x4 pd[2][2], ds[2][2];   // [tile][half]
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int qt = 2 * c + half;
      const int qb = qt * 16 + 4 * g;   // rows qb + i of this lane's registers
      const float4 ls4 = *reinterpret_cast<const float4*>(lse_s + qb);
      const float4 dl4 = *reinterpret_cast<const float4*>(del_s + qb);
      uint4 mw4 = make_uint4(0u, 0u, 0u, 0u);
      if (DM == 2) mw4 = *reinterpret_cast<const uint4*>(msk_s + kw * MSK_LD + qb);
      const float lsv[4] = {ls4.x, ls4.y, ls4.z, ls4.w}, dlv[4] = {dl4.x, dl4.y, dl4.z, dl4.w};
      const uint32_t mwv[4] = {mw4.x, mw4.y, mw4.z, mw4.w};
      f32x4 sv[2], dp[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) sv[t] = dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 qa = row_frag(Qimg, qt * 16 + lr, 32 * ks + 8 * g);
        const bf16x8 oa = row_frag(dOimg, qt * 16 + lr, 32 * ks + 8 * g);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          sv[t] = mfma_t<H>(qa, kf[t][ks], sv[t]);
          dp[t] = mfma(oa, vf[t][ks], dp[t]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t qm = (uint32_t)((qb + i - T) >> 31);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint32_t km = qm & kokm[t];
          const float p = __uint_as_float(__float_as_uint(exp2_fast(fmaf(sv[t][i], c2, -lsv[i]))) & km);
          float ksc;
          if constexpr (DM == 2) {
            ksc = __uint_as_float(__float_as_uint(dc.scale) &
                                  (uint32_t)((int32_t)(mwv[i] << (31 - (ksh + 16 * t))) >> 31));
          } else {
            ksc = keep_scale<DROP>(dc, (bh * T + (qb + i)) * (uint64_t)TP + key[t]);
          }
          pd[t][half][i] = p * ksc;
          ds[t][half][i] = p * (dp[t][i] * ksc - dlv[i]);
        }
      }
    }
    bf16x8 bp[2], bs[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bp[t] = pack_acc(pd[t][0], pd[t][1]);
      bs[t] = pack_acc(ds[t][0], ds[t][1]);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const bf16x8 ot = tr_frag(dOimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr);
      const bf16x8 qtr = to_b16<H>(tr_frag(Qimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr));
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        dv[t][dt] = mfma(ot, bp[t], dv[t][dt]);
        dk[t][dt] = mfma(qtr, bs[t], dk[t][dt]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (key[t] < T) {
      const int64_t r = (row0 + key[t]) * ld + h * DH;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store_out(dqkv, dqkv16, r + D + dt * 16 + 4 * g, dk[t][dt], scale);
        store_out(dqkv, dqkv16, r + 2 * D + dt * 16 + 4 * g, dv[t][dt], 1.f);
      }
    }
  }
}

// --------------------------------------------------------------------------------------- backward dQ
// Runs BEFORE the dK/dV kernel: delta[q] = sum_key P_d dP_d is formed here from the very P and dP
// the kernel recomputes (not as dO . O from the rounded bf16 O), so sum_key dS = 0 holds to fp32
// rounding — otherwise the residual feeds a systematic, Q-correlated error into dK. Pass 1 keeps
// P and dP*keep in registers, pass 2 forms dS and dQ^T += K^T dS^T. One workgroup per (batch, head,
// 128 queries): K and V staged once, 4 waves x query tiles w and w + 4.
template <int DM, bool H, int TM, bool T1 = false>   // DM 0: no dropout, 1: hash, 2: keep bits in memory; H: fp16 qkv; T1: T > TM - 16
__global__ void __launch_bounds__(256) attn16_bwd_dq_k(const uint16_t* __restrict__ qkv, float* __restrict__ delta,
                                                       const uint16_t* __restrict__ dO16, const float* __restrict__ lse2,
                                                       float* __restrict__ dqkv, uint16_t* __restrict__ dqkv16, int T,
                                                       int nh, float scale, DropCfg dc,
                                                       const uint32_t* __restrict__ maskw) {
  constexpr bool DROP = DM != 0;
  dc.seed = b2p_seed_eff(dc.seed, dc.epoch);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqh = (T + FWD_QB - 1) / FWD_QB;
  const int bhi = blockIdx.x / nqh, qh = blockIdx.x - bhi * nqh;
  const int b = bhi / nh, h = bhi - b * nh;
  const int D = nh * DH;
  const int64_t ld = 3 * (int64_t)D;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, lr = l & 15, g = l >> 4;
  const int64_t row0 = (int64_t)b * T;
  if (b2p_gated_off(dc.gate)) {   // LayerDrop: zero dQ (the bias reduction reads it)
    for (int half = 0; half < FWD_QB / 64; ++half) zero_block(dqkv, dqkv16, row0, qh * FWD_QB + 64 * half, T, ld, h * DH, tid);
    return;
  }
  static_assert(TM == TMAX || DM != 2, "the stored keep mask covers T <= 256");
  load_image<TM>(smem, qkv, row0, T, ld, D + h * DH, tid);                        // K (as stored: S = Q K^T)
  load_image_b16<H, TM>(smem + TM * 128, qkv, row0, T, ld, 2 * D + h * DH, tid);  // V in bf16 (dP = dO V^T)
  __syncthreads();
  const float c2 = scale * LOG2E;
  const int TP = T + (T & 1);
  const int qt0 = qh * (FWD_QB / 16) + w;
  uint32_t tailm[4];   // T1: validity masks of this lane's keys in the last key tile
#pragma unroll
  for (int i = 0; i < 4; ++i) tailm[i] = (uint32_t)((TM - 16 + 4 * g + i - T) >> 31);
  for (int qt = qt0; qt < qt0 + FWD_QB / 16 && qt * 16 < T; qt += 4) {
    uint32_t obase = 0;   // opaque image bases: no hoisting of the unrolled body's LDS addresses
    asm volatile("" : "+v"(obase));
    const char* Kimg = smem + obase;
    const char* Vimg = smem + TM * 128 + obase;
    const int q = qt * 16 + lr;
    const bool qok = q < T;
    bf16x8 qf[2], df[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[ks] = df[ks] = bf16x8{};
      if (qok) {
        qf[ks] = gload8(qkv + (row0 + q) * ld + h * DH + 32 * ks + 8 * g);
        df[ks] = gload8(dO16 + (row0 + q) * D + h * DH + 32 * ks + 8 * g);
      }
    }
    const int64_t rowc = ((int64_t)b * nh + h) * T + (qok ? q : 0);
    const float ls = qok ? lse2[rowc] : 0.f;
    const uint64_t rowidx = (uint64_t)rowc * (uint64_t)TP;
    if constexpr (TM > TMAX) {
      // T' > 256: the per-key P / dP*keep of 32 key tiles do not fit in registers beside the rest, so pass 1
      // forms delta and pass 2 recomputes S and dP per 32-key chunk (6 -> 10 MFMAs per key tile)
      auto sdp = [&](int kt, f32x4& p4, f32x4& pd4) __attribute__((always_inline)) {
        f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sv = mfma_t<H>(row_frag(Kimg, kt * 16 + lr, 32 * ks + 8 * g), qf[ks], sv);
          dp = mfma(row_frag(Vimg, kt * 16 + lr, 32 * ks + 8 * g), df[ks], dp);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = kt * 16 + 4 * g + i;
          const bool ok = qok && key < T;
          p4[i] = ok ? exp2_fast(fmaf(sv[i], c2, -ls)) : 0.f;
          pd4[i] = ok ? dp[i] * keep_scale<DROP>(dc, rowidx + key) : 0.f;
        }
      };
      float dl = 0.f;
#pragma unroll 2
      for (int kt = 0; kt < TM / 16; ++kt) {
        f32x4 p4, pd4;
        sdp(kt, p4, pd4);
#pragma unroll
        for (int i = 0; i < 4; ++i) dl += p4[i] * pd4[i];
      }
      dl += __shfl_xor(dl, 16, 64);
      dl += __shfl_xor(dl, 32, 64);
      if (qok && g == 0) delta[rowc] = dl;
      f32x4 dq[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int c = 0; c < TM / 32; ++c) {
        f32x4 ds[2];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          f32x4 p4, pd4;
          sdp(2 * c + half, p4, pd4);
#pragma unroll
          for (int i = 0; i < 4; ++i) ds[half][i] = p4[i] * (pd4[i] - dl);
        }
        const bf16x8 bs = pack_acc(ds[0], ds[1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          dq[dt] = mfma(to_b16<H>(tr_frag(Kimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr)), bs, dq[dt]);
      }
      if (qok) {
        const int64_t r = (row0 + q) * ld + h * DH;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) store_out(dqkv, dqkv16, r + dt * 16 + 4 * g, dq[dt], scale);
      }
      continue;
    }
    // keys >= T are masked; rows q >= T need no mask (a lane's dS only reaches its own, unstored dQ row)
    uint2 mw = make_uint2(0u, 0u);   // this lane's keep bytes of the query row (keys kt*16 + 4g + i)
    if (DM == 2 && qok) mw = *reinterpret_cast<const uint2*>(maskw + (int64_t)rowc * 8 + 2 * g);
    f32x4 P[16], PD[16];
    float dl = 0.f;
#pragma unroll
    for (int kt = 0; kt < 16; ++kt) {
      f32x4 sv = f32x4{0.f, 0.f, 0.f, 0.f}, dp = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        sv = mfma_t<H>(row_frag(Kimg, kt * 16 + lr, 32 * ks + 8 * g), qf[ks], sv);
        dp = mfma(row_frag(Vimg, kt * 16 + lr, 32 * ks + 8 * g), df[ks], dp);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // validity and keep as all-ones / zero bit masks formed arithmetically: compare-and-select per
        // element left 64 lane masks live in SGPR pairs across the unrolled tiles (238 SGPR spills)
        const int key = kt * 16 + 4 * g + i;
        // T1: only the last key tile holds keys >= T (its 4 masks computed once per kernel)
        const uint32_t km = T1 ? (kt == 15 ? tailm[i] : ~0u) : (uint32_t)((key - T) >> 31);
        const float p = __uint_as_float(__float_as_uint(exp2_fast(fmaf(sv[i], c2, -ls))) & km);
        float kp;
        if constexpr (DM == 2) {
          const uint32_t wd = kt < 8 ? mw.x : mw.y;
          const int bit = 8 * ((kt >> 1) & 3) + 4 * (kt & 1) + i;
          kp = __uint_as_float(__float_as_uint(dc.scale) & (uint32_t)__builtin_amdgcn_sbfe((int)wd, bit, 1));
        } else {
          kp = keep_scale<DROP>(dc, rowidx + key);
        }
        const float pd = __uint_as_float(__float_as_uint(dp[i] * kp) & km);
        P[kt][i] = p;
        PD[kt][i] = pd;
        dl += p * pd;
      }
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    if (qok && g == 0) delta[rowc] = dl;
    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float dqs = scale;
    if constexpr (H) {
      // fp16 K (as staged) x fp16 dS: the whole row's dS is in registers, so it is scaled by a power of
      // two that puts the row's largest |dS| in [1, 2) (fp16 then holds it with 11 significant bits,
      // bf16 would keep 8) and the product is unscaled at the store; no per-chunk fp16 -> bf16
      // conversion of the K^T operand
      float mx = 0.f;
#pragma unroll
      for (int kt = 0; kt < 16; ++kt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float d = P[kt][i] * (PD[kt][i] - dl);
          P[kt][i] = d;
          mx = fmaxf(mx, fabsf(d));
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const int em = min(max((int)(__float_as_uint(mx) >> 23), 1), 253);   // mx = 2^(em-127) * 1.f
      const float rs = __uint_as_float((uint32_t)(254 - em) << 23);          // 2^-(em-127)
      dqs = scale * __uint_as_float((uint32_t)em << 23);                     // scale * 2^(em-127)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        f32x4 ds[2];
#pragma unroll
        for (int half = 0; half < 2; ++half)
#pragma unroll
          for (int i = 0; i < 4; ++i) ds[half][i] = P[2 * c + half][i] * rs;
        const bf16x8 bs = pack_acc_t<true>(ds[0], ds[1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          dq[dt] = mfma_t<true>(tr_frag(Kimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr), bs, dq[dt]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        f32x4 ds[2];
#pragma unroll
        for (int half = 0; half < 2; ++half)
#pragma unroll
          for (int i = 0; i < 4; ++i) ds[half][i] = P[2 * c + half][i] * (PD[2 * c + half][i] - dl);
        const bf16x8 bs = pack_acc(ds[0], ds[1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
          dq[dt] = mfma(tr_frag(Kimg, 32 * c + 4 * g, 32 * c + 16 + 4 * g, dt * 16, lr), bs, dq[dt]);
      }
    }
    if (qok) {
      const int64_t r = (row0 + q) * ld + h * DH;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store_out(dqkv, dqkv16, r + dt * 16 + 4 * g, dq[dt], dqs);
    }
  }
}

DropCfg drop_cfg(float p, uint64_t seed) {
  DropCfg d;
  d.epoch = b2p_seed_epoch();
  d.gate = b2p_gate();
  d.seed = seed;
  d.thr = b2p_dropout_threshold(p);
  d.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  return d;
}
template <int TM>
constexpr size_t fwd_lds() { return 2 * TM * 128; }
template <int TM>
constexpr size_t bwd_lds() { return 2 * TM * 128 + 2 * TM * 4 + (TM == TMAX ? 4 * MSK_LD * 4 : 0); }

template <typename K>
int set_lds(K kern, size_t bytes) {
  B2P_CHECK_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return 0;
}
template <bool H, int TM>
int init_attrs_t() {
  int rc = 0;
  rc |= set_lds(attn16_fwd_k<0, H, TM>, fwd_lds<TM>());
  rc |= set_lds(attn16_fwd_k<1, H, TM>, fwd_lds<TM>());
  rc |= set_lds(attn16_bwd_dkv_k<0, H, TM>, bwd_lds<TM>());
  rc |= set_lds(attn16_bwd_dkv_k<1, H, TM>, bwd_lds<TM>());
  rc |= set_lds(attn16_bwd_dkv2_k<0, H, TM>, bwd_lds<TM>());
  rc |= set_lds(attn16_bwd_dkv2_k<1, H, TM>, bwd_lds<TM>());
  rc |= set_lds(attn16_bwd_dq_k<0, H, TM>, fwd_lds<TM>());
  rc |= set_lds(attn16_bwd_dq_k<1, H, TM>, fwd_lds<TM>());
  if constexpr (TM == TMAX) {
    rc |= set_lds(attn16_fwd_k<0, H, TM, true>, fwd_lds<TM>());
    rc |= set_lds(attn16_fwd_k<1, H, TM, true>, fwd_lds<TM>());
    rc |= set_lds(attn16_fwd_k<2, H, TM, true>, fwd_lds<TM>());
    rc |= set_lds(attn16_fwd_k<2, H, TM>, fwd_lds<TM>());
    rc |= set_lds(attn16_fwd_k<3, H, TM, true>, fwd_lds<TM>());
    rc |= set_lds(attn16_fwd_k<3, H, TM>, fwd_lds<TM>());
    rc |= set_lds(attn16_bwd_dkv_k<2, H, TM>, bwd_lds<TM>());
    rc |= set_lds(attn16_bwd_dkv2_k<2, H, TM>, bwd_lds<TM>());
    rc |= set_lds(attn16_bwd_dq_k<2, H, TM>, fwd_lds<TM>());
    rc |= set_lds(attn16_bwd_dq_k<0, H, TM, true>, fwd_lds<TM>());
    rc |= set_lds(attn16_bwd_dq_k<1, H, TM, true>, fwd_lds<TM>());
    rc |= set_lds(attn16_bwd_dq_k<2, H, TM, true>, fwd_lds<TM>());
  }
  return rc;
}
int init_attrs() {
  static int done = -1;
  if (done >= 0) return done;
  done = init_attrs_t<false, 256>() | init_attrs_t<true, 256>() | init_attrs_t<false, 512>() | init_attrs_t<true, 512>();
  return done;
}
}  // namespace

namespace {
// dK/dV kernel form: 1 = paired key tiles (default), 0 = per tile (B2P_ATTN_DKV2=0 or b2p_attn16_dkv_variant;
// A/B and the bitwise-equality test)
int g_dkv_variant = -1;
bool attn_dkv2() {
  if (g_dkv_variant < 0) g_dkv_variant = (getenv("B2P_ATTN_DKV2") && getenv("B2P_ATTN_DKV2")[0] == '0') ? 0 : 1;
  return g_dkv_variant != 0;
}
bool attn_t1() {   // B2P_ATTN_T1=0: the masked form for every T (A/B)
  static const bool on = !(getenv("B2P_ATTN_T1") && getenv("B2P_ATTN_T1")[0] == '0');
  return on;
}
int attn16_fwd_launch(bool half, const void* qkv16, void* O16, void* Ob16, float* lse2, int64_t B, int64_t T,
                      int64_t nh, int64_t dh, float scale, float drop_p, uint64_t drop_seed, uint32_t* mask,
                      b2p_stream_t stream, bool mask_in = false) {
  B2P_CHECK_ARG(qkv16 && O16 && lse2, "attn16_fwd: NULL pointer");
  B2P_CHECK_ARG(dh == DH && T <= 2 * TMAX && T > 0, "attn16_fwd: needs head size 64 and T <= 512");
  B2P_CHECK_ARG(!mask || T <= TMAX, "attn16_fwd: the stored keep mask covers T <= 256 (pass NULL: the backward rehashes)");
  if (B <= 0) return 0;
  if (init_attrs()) return 2;
  B2P_CHECK_ARG(B * nh * T * (T + (T & 1)) < (1ll << 32), "attn16_fwd: B * heads * T * T must stay below 2^32 "
                "(32-bit dropout element index)");
  dim3 grid((unsigned)(B * nh * ((T + FWD_QB - 1) / FWD_QB)));
  const DropCfg dc = drop_cfg(drop_p, drop_seed);
  B2P_CHECK_ARG(!mask_in || (mask && drop_p > 0.f), "attn16_fwd: reading the keep bits needs the mask and p > 0");
  const int dm = drop_p > 0.f ? (mask ? (mask_in ? 3 : 2) : 1) : 0;
  auto run = [&](auto dmc, auto hc) {
    constexpr int DM = decltype(dmc)::value;
    constexpr bool HH = decltype(hc)::value;
    if (T <= TMAX && T > TMAX - 16 && attn_t1())
      hipLaunchKernelGGL((attn16_fwd_k<DM, HH, TMAX, true>), grid, dim3(FWD_NT), fwd_lds<TMAX>(), (hipStream_t)stream,
                         (const uint16_t*)qkv16, (uint16_t*)O16, (uint16_t*)Ob16, lse2, (int)T, (int)nh, scale, dc,
                         dm >= 2 ? mask : (uint32_t*)nullptr);
    else if (T <= TMAX)
      hipLaunchKernelGGL((attn16_fwd_k<DM, HH, TMAX>), grid, dim3(FWD_NT), fwd_lds<TMAX>(), (hipStream_t)stream,
                         (const uint16_t*)qkv16, (uint16_t*)O16, (uint16_t*)Ob16, lse2, (int)T, (int)nh, scale, dc,
                         dm >= 2 ? mask : (uint32_t*)nullptr);
    else if constexpr (DM < 2)
      hipLaunchKernelGGL((attn16_fwd_k<DM, HH, 2 * TMAX>), grid, dim3(FWD_NT), fwd_lds<2 * TMAX>(), (hipStream_t)stream,
                         (const uint16_t*)qkv16, (uint16_t*)O16, (uint16_t*)Ob16, lse2, (int)T, (int)nh, scale, dc,
                         (uint32_t*)nullptr);
  };
  using F = std::false_type;
  using Tr = std::true_type;
  if (half) {
    if (dm == 3) run(std::integral_constant<int, 3>(), Tr());
    else if (dm == 2) run(std::integral_constant<int, 2>(), Tr());
    else if (dm == 1) run(std::integral_constant<int, 1>(), Tr());
    else run(std::integral_constant<int, 0>(), Tr());
  } else {
    if (dm == 3) run(std::integral_constant<int, 3>(), F());
    else if (dm == 2) run(std::integral_constant<int, 2>(), F());
    else if (dm == 1) run(std::integral_constant<int, 1>(), F());
    else run(std::integral_constant<int, 0>(), F());
  }
  B2P_CHECK_LAUNCH();
  return 0;
}
}  // namespace

extern "C" int b2p_attn16_fwd(const void* qkv16, void* O16, float* lse2, int64_t B, int64_t T, int64_t nh,
                              int64_t dh, float scale, float drop_p, uint64_t drop_seed, uint32_t* mask,
                              b2p_stream_t stream) {
  return attn16_fwd_launch(false, qkv16, O16, nullptr, lse2, B, T, nh, dh, scale, drop_p, drop_seed, mask, stream);
}

extern "C" int b2p_attn16_fwd_f16(const void* qkv16h, void* O16h, void* Ob16, float* lse2, int64_t B, int64_t T,
                                  int64_t nh, int64_t dh, float scale, float drop_p, uint64_t drop_seed,
                                  uint32_t* mask, b2p_stream_t stream) {
  return attn16_fwd_launch(true, qkv16h, O16h, Ob16, lse2, B, T, nh, dh, scale, drop_p, drop_seed, mask, stream);
}

extern "C" int b2p_attn16_fwd_keep(const void* qkv16, void* O16, float* lse2, int64_t B, int64_t T, int64_t nh,
                                   int64_t dh, float scale, float drop_p, const uint32_t* mask, b2p_stream_t stream) {
  return attn16_fwd_launch(false, qkv16, O16, nullptr, lse2, B, T, nh, dh, scale, drop_p, 0, const_cast<uint32_t*>(mask),
                           stream, true);
}

extern "C" int b2p_attn16_fwd_f16_keep(const void* qkv16h, void* O16h, void* Ob16, float* lse2, int64_t B, int64_t T,
                                       int64_t nh, int64_t dh, float scale, float drop_p, const uint32_t* mask,
                                       b2p_stream_t stream) {
  return attn16_fwd_launch(true, qkv16h, O16h, Ob16, lse2, B, T, nh, dh, scale, drop_p, 0, const_cast<uint32_t*>(mask),
                           stream, true);
}

extern "C" int b2p_attn16_keep_masks(uint32_t* mask, const uint64_t* seeds, int64_t n_layers, int64_t B, int64_t T,
                                     int64_t nh, float drop_p, b2p_stream_t stream) {
  B2P_CHECK_ARG(mask && seeds, "attn16_keep_masks: NULL pointer");
  B2P_CHECK_ARG(T > 0 && T <= TMAX && drop_p > 0.f && drop_p < 1.f, "attn16_keep_masks: needs 0 < T <= 256, 0 < p < 1");
  B2P_CHECK_ARG(B * nh * T * (T + (T & 1)) < (1ll << 32), "attn16_keep_masks: B * heads * T * T must stay below 2^32");
  const int64_t rows = B * nh * T;
  if (rows <= 0 || n_layers <= 0) return 0;
  const uint32_t thr = b2p_dropout_threshold(drop_p);
  for (int64_t l0 = 0; l0 < n_layers; l0 += KEEP_LAYERS) {
    const int nl = (int)(n_layers - l0 < KEEP_LAYERS ? n_layers - l0 : KEEP_LAYERS);
    KeepSeeds ks{};
    for (int j = 0; j < nl; ++j) ks.seed[j] = seeds[l0 + j];
    // 24 KB of (unused) LDS per workgroup: a workgroup cannot land on a CU that holds a GRU recurrence
    // (gru16: ~149 KB of its 160 KB), which it would slow by sharing its issue slots (measured: +97 us
    // on a 479 us gru16_fwd at the base workload with no LDS request)
    hipLaunchKernelGGL(attn_keep_k, dim3((unsigned)((rows * 4 * nl + 255) / 256)), dim3(256), KEEP_LDS, (hipStream_t)stream,
                       mask + l0 * rows * 8, ks, b2p_seed_epoch(), rows, (int)T, thr, nl);
    B2P_CHECK_LAUNCH();
  }
  return 0;
}

namespace {
int attn16_bwd_launch(bool half, const void* qkv16, const void* dO16, const float* lse2, float* delta_ws, float* dqkv,
                      void* dqkv16, int64_t B, int64_t T, int64_t nh, int64_t dh, float scale, float drop_p,
                      uint64_t drop_seed, const uint32_t* mask, b2p_stream_t stream) {
  B2P_CHECK_ARG(qkv16 && dO16 && lse2 && delta_ws && (dqkv || dqkv16), "attn16_bwd: NULL pointer");
  B2P_CHECK_ARG(dh == DH && T <= 2 * TMAX && T > 0, "attn16_bwd: needs head size 64 and T <= 512");
  B2P_CHECK_ARG(!mask || T <= TMAX, "attn16_bwd: the stored keep mask covers T <= 256");
  if (B <= 0) return 0;
  if (init_attrs()) return 2;
  const dim3 grid_q((unsigned)(B * nh * ((T + FWD_QB - 1) / FWD_QB)));
  const dim3 grid_k((unsigned)(B * nh * ((T + BWD_KB - 1) / BWD_KB)));
  const DropCfg dc = drop_cfg(drop_p, drop_seed);
  hipStream_t st = (hipStream_t)stream;
  const uint16_t *q = (const uint16_t*)qkv16, *d = (const uint16_t*)dO16;
  uint16_t* d16 = (uint16_t*)dqkv16;
  auto run = [&](auto dm, auto hc) {
    constexpr int DM = decltype(dm)::value;
    constexpr bool HH = decltype(hc)::value;
    if (T <= TMAX) {
      if (T > TMAX - 16 && attn_t1())
        hipLaunchKernelGGL((attn16_bwd_dq_k<DM, HH, TMAX, true>), grid_q, dim3(256), fwd_lds<TMAX>(), st, q, delta_ws,
                           d, lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
      else
        hipLaunchKernelGGL((attn16_bwd_dq_k<DM, HH, TMAX>), grid_q, dim3(256), fwd_lds<TMAX>(), st, q, delta_ws, d,
                           lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
      if (attn_dkv2())
        hipLaunchKernelGGL((attn16_bwd_dkv2_k<DM, HH, TMAX>), grid_k, dim3(256), bwd_lds<TMAX>(), st, q, delta_ws, d,
                           lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
      else
        hipLaunchKernelGGL((attn16_bwd_dkv_k<DM, HH, TMAX>), grid_k, dim3(256), bwd_lds<TMAX>(), st, q, delta_ws, d,
                           lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
    } else if constexpr (DM != 2) {
      hipLaunchKernelGGL((attn16_bwd_dq_k<DM, HH, 2 * TMAX>), grid_q, dim3(256), fwd_lds<2 * TMAX>(), st, q, delta_ws,
                         d, lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
      if (attn_dkv2())
        hipLaunchKernelGGL((attn16_bwd_dkv2_k<DM, HH, 2 * TMAX>), grid_k, dim3(256), bwd_lds<2 * TMAX>(), st, q,
                           delta_ws, d, lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
      else
        hipLaunchKernelGGL((attn16_bwd_dkv_k<DM, HH, 2 * TMAX>), grid_k, dim3(256), bwd_lds<2 * TMAX>(), st, q,
                           delta_ws, d, lse2, dqkv, d16, (int)T, (int)nh, scale, dc, mask);
    }
  };
  auto by_dm = [&](auto hc) {
    if (drop_p > 0.f && mask) run(std::integral_constant<int, 2>(), hc);
    else if (drop_p > 0.f) run(std::integral_constant<int, 1>(), hc);
    else run(std::integral_constant<int, 0>(), hc);
  };
  if (half) by_dm(std::true_type());
  else by_dm(std::false_type());
  B2P_CHECK_LAUNCH();
  return 0;
}
}  // namespace

extern "C" int b2p_attn16_dkv_variant(int v) {
  g_dkv_variant = v ? 1 : 0;
  return 0;
}

extern "C" int b2p_attn16_bwd(const void* qkv16, const void* dO16, const float* lse2, float* delta_ws, float* dqkv,
                              void* dqkv16, int64_t B, int64_t T, int64_t nh, int64_t dh, float scale, float drop_p,
                              uint64_t drop_seed, const uint32_t* mask, b2p_stream_t stream) {
  return attn16_bwd_launch(false, qkv16, dO16, lse2, delta_ws, dqkv, dqkv16, B, T, nh, dh, scale, drop_p, drop_seed,
                           mask, stream);
}

extern "C" int b2p_attn16_bwd_f16(const void* qkv16h, const void* dO16, const float* lse2, float* delta_ws,
                                  float* dqkv, void* dqkv16, int64_t B, int64_t T, int64_t nh, int64_t dh, float scale,
                                  float drop_p, uint64_t drop_seed, const uint32_t* mask, b2p_stream_t stream) {
  return attn16_bwd_launch(true, qkv16h, dO16, lse2, delta_ws, dqkv, dqkv16, B, T, nh, dh, scale, drop_p, drop_seed,
                           mask, stream);
}
