// HBM-bound kernels of the path: column reductions, dropout, LayerNorm, attention softmax,
// activation backward, front-end smoothing / col2im, weight layout transforms, weight norm.
// All fp32, float4-vectorised along the contiguous dimension where the layout allows.
#include "common.h"
#include <stdlib.h>
#include <atomic>
#include <map>
#include <mutex>
#include <utility>
#include <vector>
#include "../../include/b2p_hip.h"

namespace {
constexpr int kColsumRows = 256;  // rows per block in phase 1 (64 columns x 4 row lanes)

// part[b][blk][n] = sum_{m in block rows} f(X[b][m][n]) ; mode 0: x, 1: x*x, 2: x*Y
__global__ void __launch_bounds__(256) colsum_p1(const float* __restrict__ X, const float* __restrict__ Y,
                                                 int64_t M, int64_t N, int64_t ld, int64_t bstride, int mode,
                                                 float* __restrict__ part, int nblk) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + c;
  const int blk = blockIdx.y, b = blockIdx.z;
  const int64_t m0 = (int64_t)blk * kColsumRows;
  const int64_t m1 = m0 + kColsumRows < M ? m0 + kColsumRows : M;
  float s = 0.f;
  if (n < N) {
    const float* xp = X + b * bstride + n;
    const float* yp = (Y && mode == 2) ? Y + b * bstride + n : nullptr;
    const float yc = (Y && mode == 3) ? Y[(int64_t)b * N + n] : 0.f;
#pragma unroll 8
    for (int64_t m = m0 + rl; m < m1; m += 4) {
      const float x = xp[m * ld];
      const float dxc = x - yc;
      s += mode == 0 ? x : (mode == 1 ? x * x : (mode == 2 ? x * yp[m * ld] : dxc * dxc));
    }
  }
  red[rl][c] = s;
  __syncthreads();
  if (rl == 0 && n < N) part[((int64_t)b * nblk + blk) * N + n] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

// mode 0 with 16-B aligned rows: 128 columns (float4 per thread) x 8 row lanes per block
__global__ void __launch_bounds__(256) colsum_p1v(const float* __restrict__ X, int64_t M, int64_t N, int64_t ld,
                                                  int64_t bstride, float* __restrict__ part, int nblk) {
  __shared__ float4 red[8][32];
  const int c4 = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int64_t n = (int64_t)blockIdx.x * 128 + 4 * c4;
  const int blk = blockIdx.y, b = blockIdx.z;
  const int64_t m0 = (int64_t)blk * kColsumRows;
  const int64_t m1 = m0 + kColsumRows < M ? m0 + kColsumRows : M;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    const float* xp = X + b * bstride + n;
#pragma unroll 4
    for (int64_t m = m0 + rl; m < m1; m += 8) {
      const float4 x = *reinterpret_cast<const float4*>(xp + m * ld);
      s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
    }
  }
  red[rl][c4] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float4 t = red[0][c4];
#pragma unroll
    for (int r = 1; r < 8; ++r) {
      const float4 u = red[r][c4];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    *reinterpret_cast<float4*>(part + ((int64_t)b * nblk + blk) * N + n) = t;
  }
}

// 64 columns x 4 row groups per 256-thread block (the partial rows are summed 4-wide, then in LDS)
__global__ void __launch_bounds__(256) colsum_p2(const float* __restrict__ part, int nblk, int64_t N,
                                                 float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + c;
  const int b = blockIdx.y;
  float s = 0.f;
  if (n < N) {
    // four independent partial sums (loads issued together instead of one dependent chain: the
    // launches are small, ~12 blocks, so each thread's latency is the kernel's time)
    const float* p = part + (int64_t)b * nblk * N + n;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int i = rg;
    for (; i + 12 < nblk; i += 16) {
      s0 += p[(int64_t)i * N];
      s1 += p[(int64_t)(i + 4) * N];
      s2 += p[(int64_t)(i + 8) * N];
      s3 += p[(int64_t)(i + 12) * N];
    }
    for (; i < nblk; i += 4) s0 += p[(int64_t)i * N];
    s = (s0 + s1) + (s2 + s3);
  }
  red[rg][c] = s;
  __syncthreads();
  if (rg == 0 && n < N) {
    s = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    float* o = out + (int64_t)b * N + n;
    *o = accumulate ? *o + s : s;
  }
}

// ---- one-launch column sums: phase 2 folded into the last-arriving row block of each column strip.
// Every row block stores its partial row write-through (sc1), drains (vmcnt(0) + barrier) and counts
// itself in with one relaxed agent-scope atomic on its strip's counter; the block that draws nblk-1
// reads the strip's partials with sc1 loads (placement-independent: cdna_hip_programming.md §6
// Guideline 16, R1 / the counter form of the split-K hand-off), sums them in a fixed order and resets
// the counter to 0 for the next launch. Counters: a zero-initialised device pool; each launch takes a
// fresh range (host-side rotation), so launches on different streams / graph branches never share one.
// Replaces the separate colsum_p2 launch (~5 us of ramp for ~16-64 KB of partials) per reduction.
constexpr int kCtrPool = 1 << 18;
__device__ uint32_t g_colsum_ctr[kCtrPool];

typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mkres_cs(const void* p, uint64_t bytes) {
  const uint32_t n = bytes >= 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, n, 0x00020000);
}

// returns true in every thread of the block that arrived last at counter `ctr` (nblk arrivals)
__device__ __forceinline__ bool colsum_arrive(uint32_t* ctr, int nblk, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this block's sc1 partial stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (uint32_t)(nblk - 1);
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the sc1 loads below the count
  return last;
}

// colsum_p1v + fold: 128 columns x 8 row lanes per block, as colsum_p1v
__global__ void __launch_bounds__(256) colsum_fold_v(const float* __restrict__ X, int64_t M, int64_t N, int64_t ld,
                                                     int64_t bstride, float* __restrict__ part, int nblk,
                                                     float* __restrict__ out, int accumulate, uint32_t ctr0) {
  __shared__ float4 red[9][32];   // rows 0-7: the reduction; red[8][0]: the "arrived last" flag
  const int c4 = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int64_t n = (int64_t)blockIdx.x * 128 + 4 * c4;
  const int blk = blockIdx.y, b = blockIdx.z;
  const int64_t m0 = (int64_t)blk * kColsumRows;
  const int64_t m1 = m0 + kColsumRows < M ? m0 + kColsumRows : M;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    const float* xp = X + b * bstride + n;
#pragma unroll 4
    for (int64_t m = m0 + rl; m < m1; m += 8) {
      const float4 x = *reinterpret_cast<const float4*>(xp + m * ld);
      s.x += x.x; s.y += x.y; s.z += x.z; s.w += x.w;
    }
  }
  red[rl][c4] = s;
  __syncthreads();
  float* pb = part + (int64_t)b * nblk * N;
  const rsrc_t rp = mkres_cs(pb, (uint64_t)nblk * N * 4);
  if (rl == 0 && n < N) {
    float4 t = red[0][c4];
#pragma unroll
    for (int r = 1; r < 8; ++r) {
      const float4 u = red[r][c4];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, t), rp,
                                           (uint32_t)(((int64_t)blk * N + n) * 4), 0, 16);
  }
  if (!colsum_arrive(g_colsum_ctr + ctr0 + (uint32_t)b * gridDim.x + blockIdx.x, nblk,
                     reinterpret_cast<int*>(&red[8][0])))
    return;
  float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    for (int i = rl; i < nblk; i += 8) {
      const float4 u = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rp, (uint32_t)(((int64_t)i * N + n) * 4), 0, 16));
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
  }
  red[rl][c4] = t;
  __syncthreads();
  if (rl == 0 && n < N) {
    float4 v = red[0][c4];
#pragma unroll
    for (int r = 1; r < 8; ++r) {
      const float4 u = red[r][c4];
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    float4* o = reinterpret_cast<float4*>(out + (int64_t)b * N + n);
    if (accumulate) {
      const float4 w = *o;
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    *o = v;
  }
}

// colsum_p1 + fold: 64 columns x 4 row lanes per block, every mode, any alignment
__global__ void __launch_bounds__(256) colsum_fold(const float* __restrict__ X, const float* __restrict__ Y,
                                                   int64_t M, int64_t N, int64_t ld, int64_t bstride, int mode,
                                                   float* __restrict__ part, int nblk, float* __restrict__ out,
                                                   int accumulate, uint32_t ctr0) {
  __shared__ float red[5][64];    // rows 0-3: the reduction; red[4][0]: the "arrived last" flag
  const int c = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int64_t n = (int64_t)blockIdx.x * 64 + c;
  const int blk = blockIdx.y, b = blockIdx.z;
  const int64_t m0 = (int64_t)blk * kColsumRows;
  const int64_t m1 = m0 + kColsumRows < M ? m0 + kColsumRows : M;
  float s = 0.f;
  if (n < N) {
    const float* xp = X + b * bstride + n;
    const float* yp = (Y && mode == 2) ? Y + b * bstride + n : nullptr;
    const float yc = (Y && mode == 3) ? Y[(int64_t)b * N + n] : 0.f;
#pragma unroll 8
    for (int64_t m = m0 + rl; m < m1; m += 4) {
      const float x = xp[m * ld];
      const float dxc = x - yc;
      s += mode == 0 ? x : (mode == 1 ? x * x : (mode == 2 ? x * yp[m * ld] : dxc * dxc));
    }
  }
  red[rl][c] = s;
  __syncthreads();
  float* pb = part + (int64_t)b * nblk * N;
  const rsrc_t rp = mkres_cs(pb, (uint64_t)nblk * N * 4);
  if (rl == 0 && n < N)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, red[0][c] + red[1][c] + red[2][c] + red[3][c]),
                                          rp, (uint32_t)(((int64_t)blk * N + n) * 4), 0, 16);
  if (!colsum_arrive(g_colsum_ctr + ctr0 + (uint32_t)b * gridDim.x + blockIdx.x, nblk,
                     reinterpret_cast<int*>(&red[4][0])))
    return;
  float t = 0.f;
  if (n < N)
    for (int i = rl; i < nblk; i += 4)
      t += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rp, (uint32_t)(((int64_t)i * N + n) * 4), 0,
                                                                          16));
  red[rl][c] = t;
  __syncthreads();
  if (rl == 0 && n < N) {
    const float v = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    float* o = out + (int64_t)b * N + n;
    *o = accumulate ? *o + v : v;
  }
}

// Counter allocation. Every launch takes a fresh range by host-side rotation over the pool. A captured
// graph replays its launches' ranges for as long as it lives, so the ranges allocated while a capture
// records (b2p_colsum_pin_begin .. _end) stay reserved until b2p_colsum_unpin: later launches (eager,
// or another graph, possibly on a concurrent stream) skip them and never share a counter with a live
// graph. When no free range fits, the launch falls back to the two-launch form (no counter at all).
struct CtrPool {
  std::mutex mu;
  uint32_t cursor = 0;
  bool recording = false;
  int64_t next_id = 1;
  std::vector<std::pair<uint32_t, uint32_t>> rec;                            // ranges of the recording
  std::map<int64_t, std::vector<std::pair<uint32_t, uint32_t>>> pins;        // id -> reserved ranges

  // first start >= base at which [start, start + n) misses every reserved range (or kCtrPool)
  uint32_t fit(uint32_t base, uint32_t n) const {
    bool moved = true;
    while (moved && base + n <= (uint32_t)kCtrPool) {
      moved = false;
      for (const auto& kv : pins)
        for (const auto& r : kv.second)
          if (base < r.second && r.first < base + n) { base = r.second; moved = true; }
    }
    return base;
  }
  int64_t alloc(uint32_t n) {
    std::lock_guard<std::mutex> g(mu);
    uint32_t b = fit(cursor, n);
    if (b + n > (uint32_t)kCtrPool) b = fit(0, n);    // wrap once
    if (b + n > (uint32_t)kCtrPool) return -1;        // everything left is reserved by live graphs
    cursor = b + n;
    if (recording) {
      if (!rec.empty() && rec.back().second == b) rec.back().second = b + n;
      else rec.emplace_back(b, b + n);
    }
    return b;
  }
};
CtrPool& ctr_pool() {
  static CtrPool p;
  return p;
}

// first counter of a fresh range of n (n <= kCtrPool / 4), or -1 when the one-launch form is off
int64_t colsum_ctr_range(int64_t n) {
  static const bool on = [] {
    const char* e = getenv("B2P_COLSUM_FOLD");
    return !(e && e[0] == '0');
  }();
  if (!on || n > kCtrPool / 4) return -1;
  return ctr_pool().alloc((uint32_t)n);
}

}  // namespace

namespace {
struct I64Vals {
  int64_t v[64];
};
__global__ void i64_fill_k(int64_t* __restrict__ dst, I64Vals vals, int n) {
  const int i = threadIdx.x;
  if (i < n) dst[i] = vals.v[i];
}
}  // namespace

// dst[0 .. n) = vals (n <= 64) by a kernel whose arguments carry the values: stream-ordered and
// capturable into a graph (no host-to-device copy); small index / pointer tables of batched launches
extern "C" int b2p_i64_fill(int64_t* dst, const int64_t* vals, int n, b2p_stream_t stream) {
  B2P_CHECK_ARG(dst && vals && n >= 0 && n <= 64, "i64_fill: n must be 0 .. 64 with non-NULL pointers");
  if (n == 0) return 0;
  I64Vals v;
  for (int i = 0; i < n; ++i) v.v[i] = vals[i];
  hipLaunchKernelGGL(i64_fill_k, dim3(1), dim3(64), 0, (hipStream_t)stream, dst, v, n);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_colsum_pin_begin(void) {
  CtrPool& p = ctr_pool();
  std::lock_guard<std::mutex> g(p.mu);
  B2P_CHECK_ARG(!p.recording, "colsum_pin_begin: a recording is already open");
  p.recording = true;
  p.rec.clear();
  return 0;
}

extern "C" int64_t b2p_colsum_pin_end(void) {
  CtrPool& p = ctr_pool();
  std::lock_guard<std::mutex> g(p.mu);
  if (!p.recording) { b2p_set_error("colsum_pin_end: no recording is open"); return -1; }
  p.recording = false;
  const int64_t id = p.next_id++;
  p.pins[id] = p.rec;
  p.rec.clear();
  return id;
}

extern "C" int b2p_colsum_unpin(int64_t id) {
  CtrPool& p = ctr_pool();
  std::lock_guard<std::mutex> g(p.mu);
  p.pins.erase(id);
  return 0;
}

extern "C" int64_t b2p_colsum_pool_state(int64_t set_cursor, int64_t* reserved) {
  CtrPool& p = ctr_pool();
  std::lock_guard<std::mutex> g(p.mu);
  if (set_cursor >= 0 && set_cursor < kCtrPool) p.cursor = (uint32_t)set_cursor;
  if (reserved) {
    int64_t r = 0;
    for (const auto& kv : p.pins)
      for (const auto& q : kv.second) r += q.second - q.first;
    *reserved = r;
  }
  return p.cursor;
}

// out[b][n] (+)= sum_m f(X[b][m][n]); mode 0: x, 1: x^2, 2: x*Y[b][m][n], 3: (x - Y[b][n])^2
int colsum_impl(const float* X, const float* Y, int64_t batch, int64_t M, int64_t N, int64_t ld,
                int64_t bstride, int mode, float* out, int accumulate, float* part, hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  const int nblk = (int)((M + kColsumRows - 1) / kColsumRows);
  const bool vec = mode == 0 && N % 4 == 0 && ld % 4 == 0 && bstride % 4 == 0 && ((uintptr_t)X & 15u) == 0 &&
                   ((uintptr_t)part & 15u) == 0 && ((uintptr_t)out & 15u) == 0;
  const int64_t gx = vec ? (N + 127) / 128 : (N + 63) / 64;
  const int64_t ctr0 = nblk * N < ((int64_t)1 << 30) ? colsum_ctr_range(gx * batch) : -1;
  if (ctr0 >= 0) {
    dim3 g((unsigned)gx, nblk, (unsigned)batch);
    if (vec)
      hipLaunchKernelGGL(colsum_fold_v, g, dim3(256), 0, st, X, M, N, ld, bstride, part, nblk, out, accumulate,
                         (uint32_t)ctr0);
    else
      hipLaunchKernelGGL(colsum_fold, g, dim3(256), 0, st, X, Y, M, N, ld, bstride, mode, part, nblk, out,
                         accumulate, (uint32_t)ctr0);
    B2P_CHECK_LAUNCH();
    return 0;
  }
  if (vec) {
    dim3 g1((unsigned)((N + 127) / 128), nblk, (unsigned)batch);
    hipLaunchKernelGGL(colsum_p1v, g1, dim3(256), 0, st, X, M, N, ld, bstride, part, nblk);
  } else {
    dim3 g1((unsigned)((N + 63) / 64), nblk, (unsigned)batch);
    hipLaunchKernelGGL(colsum_p1, g1, dim3(256), 0, st, X, Y, M, N, ld, bstride, mode, part, nblk);
  }
  dim3 g2((unsigned)((N + 63) / 64), (unsigned)batch);
  hipLaunchKernelGGL(colsum_p2, g2, dim3(256), 0, st, part, nblk, N, out, accumulate);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_colsum_parts(const float* part, int64_t ntiles, int64_t N, float* out, int accumulate,
                                b2p_stream_t stream) {
  B2P_CHECK_ARG(part && out, "colsum_parts: NULL pointer");
  if (N <= 0 || ntiles <= 0) return 0;
  dim3 g2((unsigned)((N + 63) / 64), 1);
  hipLaunchKernelGGL(colsum_p2, g2, dim3(256), 0, (hipStream_t)stream, part, (int)ntiles, N, out, accumulate);
  B2P_CHECK_LAUNCH();
  return 0;
}

namespace {

// y = x * (*s): a gradient scaled by the incoming scalar gradient of a reduced loss, read on the device
// (the CTC loss backward: d loss_total / d logits = grad * d loss_total / d loss)
__global__ void scale_dev_k(const float4* __restrict__ x, const float* __restrict__ s, float4* __restrict__ y,
                            int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float c = *s;
  const float4 v = x[i];
  y[i] = make_float4(v.x * c, v.y * c, v.z * c, v.w * c);
}
__global__ void scale_dev_tail_k(const float* __restrict__ x, const float* __restrict__ s, float* __restrict__ y,
                                 int64_t n0, int64_t n) {
  const int64_t i = n0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] * *s;
}

// ------------------------------------------------------------------ dropout
__global__ void dropout_k(const float* __restrict__ x, float* __restrict__ y, int64_t n, uint32_t thr,
                          float scale, uint64_t seed, const uint64_t* __restrict__ epoch) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  seed = b2p_seed_eff(seed, epoch);
  y[i] = b2p_keep(seed, (uint64_t)i, thr) ? x[i] * scale : 0.f;
}

// ------------------------------------------------------------------ LayerNorm
// one wave per row; cols <= 64 * 4 * LN_MAXV
constexpr int LN_MAXV = 4;
__global__ void __launch_bounds__(256) ln_fwd_k(const float* __restrict__ x, const float* __restrict__ gamma,
                                                const float* __restrict__ beta, float* __restrict__ y,
                                                float* __restrict__ mean, float* __restrict__ rstd,
                                                int64_t rows, int cols, float eps, uint32_t thr, float dscale,
                                                uint64_t seed, float drop_p, uint16_t* __restrict__ y16,
                                                const uint64_t* __restrict__ epoch, int y16_half = 0,
                                                uint16_t* __restrict__ y16b = nullptr) {
  seed = b2p_seed_eff(seed, epoch);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = cols >> 2;
  const float4* xr = reinterpret_cast<const float4*>(x + row * cols);
  float4 v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) { v[i] = xr[c]; s += v[i].x + v[i].y + v[i].z + v[i].w; }
  }
  const float mu = warp_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
      const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
      q += a * a + b * b + cc * cc + d * d;
    }
  }
  const float var = warp_sum(q) / cols;
  const float rs = rsqrtf(var + eps);
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  const float4* b4 = reinterpret_cast<const float4*>(beta);
  float4* yr = reinterpret_cast<float4*>(y + row * cols);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
      const float4 g = g4[c], bb = b4[c];
      float4 o;
      o.x = (v[i].x - mu) * rs * g.x + bb.x;
      o.y = (v[i].y - mu) * rs * g.y + bb.y;
      o.z = (v[i].z - mu) * rs * g.z + bb.z;
      o.w = (v[i].w - mu) * rs * g.w + bb.w;
      if (drop_p > 0.f) {
        const uint64_t base = (uint64_t)row * cols + 4 * c;
        bool kk[4];
        b2p_keep4(seed, base, thr, kk);   // base % 4 == 0
        o.x = kk[0] ? o.x * dscale : 0.f;
        o.y = kk[1] ? o.y * dscale : 0.f;
        o.z = kk[2] ? o.z * dscale : 0.f;
        o.w = kk[3] ? o.w * dscale : 0.f;
      }
      if (y) yr[c] = o;
      if (y16) reinterpret_cast<uint2*>(y16 + row * cols)[c] = b2p_pack16x4(o, y16_half);
      if (y16b) reinterpret_cast<uint2*>(y16b + row * cols)[c] = b2p_pack_bf16x4(o);
    }
  }
}

// LayerNorm + rotary embedding in one pass (the Conformer attention block's input: Q/K read the rotated
// LN output, V the plain one), 16-bit outputs only: h16 / hr16 (the forward GEMM operands, fp16 when
// half) and h16b / hr16b (bf16 copies, the backward's weight-gradient operands; a null pointer skips a
// copy). Lane l holds float4 c = l + 64 i; within a head of HD columns the rotate-half partner of
// columns 4c .. 4c+3 is float4 c ^ (HD / 8), i.e. lane l ^ (HD / 8) of the same i (HD / 4 divides 64).
// The LayerNorm and rotation arithmetic is that of ln_fwd_k and rotary16_k (conformer.hip), so the
// outputs equal LN -> fp32 -> rotary16 bit for bit. TF conf Wav2Vec2ConformerRotaryPositionalEmbedding
// / Wav2Vec2ConformerSelfAttention (rotary on the LN output for query and key only).
template <int HD>
__global__ void __launch_bounds__(256) ln_rot16_k(const float* __restrict__ x, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, float* __restrict__ mean,
                                                  float* __restrict__ rstd, int64_t rows, int cols, float eps, int T,
                                                  const float* __restrict__ ct, const float* __restrict__ st,
                                                  int half16, uint16_t* __restrict__ h16, uint16_t* __restrict__ h16b,
                                                  uint16_t* __restrict__ hr16, uint16_t* __restrict__ hr16b) {
  static_assert(HD % 8 == 0 && 64 % (HD / 4) == 0, "head dim: the partner float4 must sit in the same wave row");
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;   // wave-uniform: the shuffles below see whole waves only
  const int nv = cols >> 2;
  const float4* xr = reinterpret_cast<const float4*>(x + row * cols);
  float4 v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) { v[i] = xr[c]; s += v[i].x + v[i].y + v[i].z + v[i].w; }
  }
  const float mu = warp_sum(s) / cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
      const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
      q += a * a + b * b + cc * cc + d * d;
    }
  }
  const float var = warp_sum(q) / cols;
  const float rs = rsqrtf(var + eps);
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  const float4* b4 = reinterpret_cast<const float4*>(beta);
  const int t = (int)(row % T);
  const int d = (4 * lane) % HD;           // head-local column of this lane's float4 (same for every i)
  const float sg = d < HD / 2 ? -1.f : 1.f;
  const float4 cs = *reinterpret_cast<const float4*>(ct + (int64_t)t * HD + d);
  const float4 sn = *reinterpret_cast<const float4*>(st + (int64_t)t * HD + d);
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (64 * i < nv) {   // uniform over the wave (nv % 64 == 0 is checked on the host): shuffles stay whole
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (c < nv) {
        const float4 g = g4[c], bb = b4[c];
        o.x = (v[i].x - mu) * rs * g.x + bb.x;
        o.y = (v[i].y - mu) * rs * g.y + bb.y;
        o.z = (v[i].z - mu) * rs * g.z + bb.z;
        o.w = (v[i].w - mu) * rs * g.w + bb.w;
      }
      float4 ov;
      ov.x = __shfl_xor(o.x, HD / 8);
      ov.y = __shfl_xor(o.y, HD / 8);
      ov.z = __shfl_xor(o.z, HD / 8);
      ov.w = __shfl_xor(o.w, HD / 8);
      float4 r;
      r.x = o.x * cs.x + sg * ov.x * sn.x;
      r.y = o.y * cs.y + sg * ov.y * sn.y;
      r.z = o.z * cs.z + sg * ov.z * sn.z;
      r.w = o.w * cs.w + sg * ov.w * sn.w;
      const int64_t off = row * cols;
      if (h16) reinterpret_cast<uint2*>(h16 + off)[c] = b2p_pack16x4(o, half16);
      if (h16b) reinterpret_cast<uint2*>(h16b + off)[c] = b2p_pack_bf16x4(o);
      if (hr16) reinterpret_cast<uint2*>(hr16 + off)[c] = b2p_pack16x4(r, half16);
      if (hr16b) reinterpret_cast<uint2*>(hr16b + off)[c] = b2p_pack_bf16x4(r);
    }
  }
}

constexpr int LN_BWD_ROWS = 16;   // rows per block (4 per wave): ~500 blocks at 8k rows
// PF: prefetch the next row (B2P_LN_PREFETCH, default 1). MODE bits: 1 = dx_accum, 2 = dx_accum2, 4 = dxd
// (compile-time, so a form holds registers only for the streams it reads: all three at once would not
// fit two waves per SIMD)
constexpr int LNB_A1 = 1, LNB_A2 = 2, LNB_DXD = 4;
template <bool PF, int MODE>
__global__ void __launch_bounds__(256) ln_bwd_k(const float* __restrict__ dy, const float* __restrict__ x,
                                                const float* __restrict__ gamma, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, float* __restrict__ dx,
                                                const float* __restrict__ dx_accum, float* __restrict__ part,
                                                int64_t rows, int cols, uint32_t thr, float dscale, uint64_t seed,
                                                float drop_p, float* __restrict__ dxd, uint32_t thr2, float dscale2,
                                                uint64_t seed2, uint16_t* __restrict__ d16, const uint64_t* __restrict__ epoch,
                                                const float* __restrict__ dx_accum2) {
  seed = b2p_seed_eff(seed, epoch);
  seed2 = b2p_seed_eff(seed2, epoch);
  __shared__ float red[4][3][LN_MAXV * 256];   // cols <= 1024
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = cols >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(gamma);
  float4 dg[LN_MAXV], db[LN_MAXV], dd[LN_MAXV];
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    dg[i] = make_float4(0, 0, 0, 0); db[i] = make_float4(0, 0, 0, 0); dd[i] = make_float4(0, 0, 0, 0);
  }
  // software-pipelined rows: row rr+1's dy / x are in flight while row rr is reduced and written
  // (one wave per row: without the prefetch each row paid a full load latency before any math)
  const int64_t row_base = (int64_t)blockIdx.x * LN_BWD_ROWS + wave * (LN_BWD_ROWS / 4);
  // the residual gradient dx_accum is fetched with dy / x (read at the store, it cost a full load
  // latency per row)
  float4 nd[LN_MAXV], nx[LN_MAXV], na[LN_MAXV], nb[LN_MAXV];
  auto fetch = [&](int64_t r) {
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < nv && r < rows) {
        nd[i] = reinterpret_cast<const float4*>(dy + r * cols)[c];
        nx[i] = reinterpret_cast<const float4*>(x + r * cols)[c];
        if (MODE & LNB_A1) na[i] = reinterpret_cast<const float4*>(dx_accum + r * cols)[c];
        if (MODE & LNB_A2) nb[i] = reinterpret_cast<const float4*>(dx_accum2 + r * cols)[c];
      }
    }
  };
  fetch(row_base);
  float4 gk[LN_MAXV];   // gamma, loaded once per wave (was re-read for every row)
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) gk[i] = g4[c];
  }
  for (int rr = 0; rr < LN_BWD_ROWS / 4; ++rr) {
    const int64_t row = row_base + rr;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    if (!PF && rr > 0) fetch(row);
    float4 cd[LN_MAXV], cx[LN_MAXV], ca[LN_MAXV], cb[LN_MAXV];
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      cd[i] = nd[i];
      cx[i] = nx[i];
      ca[i] = na[i];
      cb[i] = nb[i];
    }
    if (PF && rr + 1 < LN_BWD_ROWS / 4) fetch(row + 1);
    float4 xh[LN_MAXV], gg[LN_MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < nv) {
        float4 d = cd[i];
        if (drop_p > 0.f) {
          const uint64_t base = (uint64_t)row * cols + 4 * c;
          bool kk[4];
          b2p_keep4(seed, base, thr, kk);   // base % 4 == 0
          d.x = kk[0] ? d.x * dscale : 0.f;
          d.y = kk[1] ? d.y * dscale : 0.f;
          d.z = kk[2] ? d.z * dscale : 0.f;
          d.w = kk[3] ? d.w * dscale : 0.f;
        }
        const float4 xv = cx[i], g = gk[i];
        xh[i] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
        gg[i] = make_float4(d.x * g.x, d.y * g.y, d.z * g.z, d.w * g.w);
        s1 += gg[i].x + gg[i].y + gg[i].z + gg[i].w;
        s2 += gg[i].x * xh[i].x + gg[i].y * xh[i].y + gg[i].z * xh[i].z + gg[i].w * xh[i].w;
        dg[i].x += d.x * xh[i].x; dg[i].y += d.y * xh[i].y; dg[i].z += d.z * xh[i].z; dg[i].w += d.w * xh[i].w;
        db[i].x += d.x; db[i].y += d.y; db[i].z += d.z; db[i].w += d.w;
      }
    }
    s1 = warp_sum(s1) / cols;
    s2 = warp_sum(s2) / cols;
    float4* dxr = reinterpret_cast<float4*>(dx + row * cols);
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
      const int c = lane + 64 * i;
      if (c < nv) {
        float4 o;
        o.x = rs * (gg[i].x - s1 - xh[i].x * s2);
        o.y = rs * (gg[i].y - s1 - xh[i].y * s2);
        o.z = rs * (gg[i].z - s1 - xh[i].z * s2);
        o.w = rs * (gg[i].w - s1 - xh[i].w * s2);
        if (MODE & LNB_A1) {
          // the residual add stays a separate rounding (no fused multiply-add with the rs product):
          // the same bits as when the add sat behind its own load
          asm volatile("" : "+v"(o.x), "+v"(o.y), "+v"(o.z), "+v"(o.w));
          const float4 a = ca[i];
          o.x += a.x; o.y += a.y; o.z += a.z; o.w += a.w;
        }
        float4 ox = o;
        if (MODE & LNB_A2) {   // a separate rounding after the first accumulator, as autograd's add was
          asm volatile("" : "+v"(ox.x), "+v"(ox.y), "+v"(ox.z), "+v"(ox.w));
          const float4 b = cb[i];
          ox.x += b.x; ox.y += b.y; ox.z += b.z; ox.w += b.w;
        }
        dxr[c] = ox;
        if (d16 && !(MODE & LNB_DXD)) reinterpret_cast<uint2*>(d16 + row * cols)[c] = b2p_pack_bf16x4(ox);
        if (MODE & LNB_DXD) {   // gradient of the dropout that produced this LN's input (residual branch)
          const uint64_t base = (uint64_t)row * cols + 4 * c;
          float4 q;
          bool kk[4];
          b2p_keep4(seed2, base, thr2, kk);   // base % 4 == 0
          q.x = kk[0] ? o.x * dscale2 : 0.f;
          q.y = kk[1] ? o.y * dscale2 : 0.f;
          q.z = kk[2] ? o.z * dscale2 : 0.f;
          q.w = kk[3] ? o.w * dscale2 : 0.f;
          reinterpret_cast<float4*>(dxd + row * cols)[c] = q;
          if (d16) reinterpret_cast<uint2*>(d16 + row * cols)[c] = b2p_pack_bf16x4(q);
          dd[i].x += q.x; dd[i].y += q.y; dd[i].z += q.z; dd[i].w += q.w;
        }
      }
    }
  }
  // block reduction of dgamma/dbeta partials
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = lane + 64 * i;
    if (c < nv) {
      reinterpret_cast<float4*>(red[wave][0])[c] = dg[i];
      reinterpret_cast<float4*>(red[wave][1])[c] = db[i];
      reinterpret_cast<float4*>(red[wave][2])[c] = dd[i];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
#pragma unroll
    for (int q = 0; q < 3; ++q)   // [3][nblk][cols]: each output's partial rows contiguous
      part[((int64_t)q * gridDim.x + blockIdx.x) * cols + c] = red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c];
  }
}

// parameter gradients of the LayerNorm backward in one launch: the [nblk][3][cols] block partials
// (dgamma | dbeta | dropout-input bias) summed over the blocks straight into their destinations (was
// the two-phase column sum + a scatter: three launches per LayerNorm backward). 128 columns (float4 per
// thread) x 8 row lanes per block, 8 independent partial sums per thread.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) ln_param_reduce_k(const float* __restrict__ part, int nblk, int cols,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         float* __restrict__ dbias_in) {
  __shared__ float4 red[8][32];
  const int c4 = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int n = blockIdx.x * 128 + 4 * c4;   // column of the [3][cols] row
  const int N = 3 * cols;
  const int q0 = n / cols;                   // output (dgamma | dbeta | dbias_in): partials [q0][nblk][cols]
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    const float* p = part + (int64_t)q0 * nblk * cols + (n - q0 * cols);
    // rows rl, rl + 8, ... summed in order; 32 of them in flight per batch (8 per batch left each thread
    // ~8 dependent memory round trips at 500 partial rows: 7.1 us per launch on the Conformer)
    // (rows past the end load as +0: adding them leaves every sum unchanged)
    for (int r = rl; r < nblk; r += 8 * 32) {
      float4 x[32];
#pragma unroll
      for (int k = 0; k < 32; ++k)
        x[k] = r + 8 * k < nblk ? *reinterpret_cast<const float4*>(p + (int64_t)(r + 8 * k) * cols)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 32; ++k) { s.x += x[k].x; s.y += x[k].y; s.z += x[k].z; s.w += x[k].w; }
    }
  }
  red[rl][c4] = s;
  __syncthreads();
  if (rl == 0 && n < N) {
    float4 t = red[0][c4];
#pragma unroll
    for (int r = 1; r < 8; ++r) {
      const float4 u = red[r][c4];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const int q = n / cols, cc = n - q * cols;   // cols % 4 == 0: a float4 never straddles two outputs
    float* dst = q == 0 ? dgamma : (q == 1 ? dbeta : dbias_in);
    if (dst) *reinterpret_cast<float4*>(dst + cc) = t;
  }
}

// ------------------------------------------------------------------ attention softmax
// one wave per row, row length n <= 64*8; dropout element index row * (n rounded up to even) + c (the
// fused attention kernels draw the same mask, csrc/attn16.hip)
constexpr int SM_MAXE = 8;
__global__ void __launch_bounds__(256) softmax_fwd_k(const float* __restrict__ S, float* __restrict__ P,
                                                     float* __restrict__ Pd, int64_t rows, int n, int64_t ld,
                                                     uint32_t thr, float dscale, uint64_t seed, float drop_p,
                                                     const uint64_t* __restrict__ epoch) {
  seed = b2p_seed_eff(seed, epoch);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* sr = S + row * ld;
  float v[SM_MAXE];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < SM_MAXE; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < n ? sr[c] : -INFINITY;
    mx = fmaxf(mx, v[i]);
  }
  mx = warp_max(mx);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < SM_MAXE; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < n ? __expf(v[i] - mx) : 0.f;
    s += v[i];
  }
  const float inv = 1.0f / warp_sum(s);
  float* pr = P + row * ld;
  float* pdr = Pd + row * ld;
#pragma unroll
  for (int i = 0; i < SM_MAXE; ++i) {
    const int c = lane + 64 * i;
    if (c < n) {
      const float p = v[i] * inv;
      pr[c] = p;
      if (drop_p > 0.f) pdr[c] = b2p_keep(seed, (uint64_t)row * (n + (n & 1)) + c, thr) ? p * dscale : 0.f;
      else pdr[c] = p;
    } else if (c < ld) {
      pr[c] = 0.f;
      pdr[c] = 0.f;
    }
  }
}

__global__ void __launch_bounds__(256) softmax_bwd_k(const float* __restrict__ P, const float* __restrict__ dPd,
                                                     float* __restrict__ dS, int64_t rows, int n, int64_t ld,
                                                     uint32_t thr, float dscale, uint64_t seed, float drop_p,
                                                     const uint64_t* __restrict__ epoch) {
  seed = b2p_seed_eff(seed, epoch);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* pr = P + row * ld;
  const float* gr = dPd + row * ld;
  float p[SM_MAXE], g[SM_MAXE];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < SM_MAXE; ++i) {
    const int c = lane + 64 * i;
    p[i] = c < n ? pr[c] : 0.f;
    float gv = c < n ? gr[c] : 0.f;
    if (drop_p > 0.f && c < n) gv = b2p_keep(seed, (uint64_t)row * (n + (n & 1)) + c, thr) ? gv * dscale : 0.f;
    g[i] = gv;
    s += p[i] * gv;
  }
  s = warp_sum(s);
  float* dr = dS + row * ld;
#pragma unroll
  for (int i = 0; i < SM_MAXE; ++i) {
    const int c = lane + 64 * i;
    if (c < n) dr[c] = p[i] * (g[i] - s);
    else if (c < ld) dr[c] = 0.f;
  }
}

__device__ __forceinline__ float act_bwd_one(float dy, float x, int act) {
  float g = 1.f;
  if (act == B2P_ACT_GELU) g = b2p_gelu_grad(x);
  else if (act == B2P_ACT_SOFTSIGN) { const float d = 1.f + fabsf(x); g = 1.f / (d * d); }
  else if (act == B2P_ACT_SILU) g = b2p_silu_grad(x);
  return dy * g;
}
__global__ void act_bwd_k(const float* __restrict__ dy, const float* __restrict__ pre, float* __restrict__ dx,
                          int64_t n, int act) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dx[i] = act_bwd_one(dy[i], pre[i], act);
}
// 4 elements per thread through 16-byte accesses (the front end's softsign' over B x L x 256: the scalar
// form ran at ~1 TB/s), same expression per element
__global__ void act_bwd4_k(const float4* __restrict__ dy, const float4* __restrict__ pre, float4* __restrict__ dx,
                           int64_t n4, int act) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const float4 d = dy[i], x = pre[i];
  dx[i] = make_float4(act_bwd_one(d.x, x.x, act), act_bwd_one(d.y, x.y, act), act_bwd_one(d.z, x.z, act),
                      act_bwd_one(d.w, x.w, act));
}

// ------------------------------------------------------------------ front-end
__global__ void gauss_k(const float* __restrict__ x, const float* __restrict__ taps, int ntaps,
                        float* __restrict__ y, int64_t B, int64_t L, int64_t C4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * L * C4) return;
  const int64_t c4 = i % C4;
  const int64_t l = (i / C4) % L;
  const int64_t b = i / (C4 * L);
  const int left = (ntaps - 1) / 2;
  const float4* xb = reinterpret_cast<const float4*>(x) + b * L * C4 + c4;
  float4 acc = make_float4(0, 0, 0, 0);
  for (int j = 0; j < ntaps; ++j) {
    const int64_t src = l + j - left;
    if (src < 0 || src >= L) continue;
    const float w = taps[j];
    const float4 v = xb[src * C4];
    acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
  }
  reinterpret_cast<float4*>(y)[i] = acc;
}

__global__ void col2im_k(const float* __restrict__ dA, const float* __restrict__ Z, float* __restrict__ dX,
                         int64_t B, int64_t L, int64_t C4, int64_t T, int ktaps, int stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * L * C4) return;
  const int64_t c4 = i % C4;
  const int64_t l = (i / C4) % L;
  const int64_t b = i / (C4 * L);
  const int64_t C = C4 * 4;
  const int64_t rowlen = (int64_t)ktaps * C;
  float4 acc = make_float4(0, 0, 0, 0);
  // taps with (l - tap) % stride == 0
  int tap0 = (int)(l % stride);
  for (int tap = tap0; tap < ktaps; tap += stride) {
    const int64_t t = (l - tap) / stride;
    if (l - tap < 0) break;
    if (t >= T) continue;
    const float4 v = reinterpret_cast<const float4*>(dA + (b * T + t) * rowlen + (int64_t)tap * C)[c4];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (Z) {
    const float4 z = reinterpret_cast<const float4*>(Z)[i];
    float d;
    d = 1.f + fabsf(z.x); acc.x /= d * d;
    d = 1.f + fabsf(z.y); acc.y /= d * d;
    d = 1.f + fabsf(z.z); acc.z /= d * d;
    d = 1.f + fabsf(z.w); acc.w /= d * d;
  }
  reinterpret_cast<float4*>(dX)[i] = acc;
}

__global__ void day_reduce_k(const float* __restrict__ ps, const int64_t* __restrict__ day, int64_t B,
                             int64_t ndays, int64_t elems, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ndays * elems) return;
  const int64_t d = i / elems, e = i % elems;
  float s = 0.f;
  for (int64_t b = 0; b < B; ++b)
    if (day[b] == d) s += ps[b * elems + e];
  out[i] = s;
}

// ------------------------------------------------------------------ weight layouts
__global__ void conv_perm_k(const float* __restrict__ in, float* __restrict__ out, int64_t O, int64_t I,
                            int64_t K, int inverse) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= O * I * K) return;
  // canonical index: (o, i, k) with k fastest in the reference layout
  const int64_t k = idx % K, i = (idx / K) % I, o = idx / (K * I);
  const int64_t ref = idx;
  const int64_t perm = o * I * K + k * I + i;
  if (inverse) out[ref] = in[perm];
  else out[perm] = in[ref];
}

// the same permutation through LDS, one output channel o per block: (I x K) <-> (K x I) transposed in
// a padded tile (row stride K + 1: conflict-free column reads), both global passes coalesced
__global__ void __launch_bounds__(256) conv_perm_tile_k(const float* __restrict__ in, float* __restrict__ out,
                                                        int I, int K, int inverse) {
  extern __shared__ float tile[];   // I * (K + 1)
  const int64_t base = (int64_t)blockIdx.x * I * K;
  const int n = I * K;
  if (!inverse) {   // in (i, k) -> out (k, i)
    for (int t = threadIdx.x; t < n; t += 256) {
      const int i = t / K, k = t - i * K;
      tile[i * (K + 1) + k] = in[base + t];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n; t += 256) {
      const int k = t / I, i = t - k * I;
      out[base + t] = tile[i * (K + 1) + k];
    }
  } else {          // in (k, i) -> out (i, k)
    for (int t = threadIdx.x; t < n; t += 256) {
      const int k = t / I, i = t - k * I;
      tile[i * (K + 1) + k] = in[base + t];
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n; t += 256) {
      const int i = t / K, k = t - i * K;
      out[base + t] = tile[i * (K + 1) + k];
    }
  }
}

// conv_perm_tile_k for power-of-two I and K (>= 4; the GRU layer-0 input weight: I = 256 channels, K = 32
// taps): 16-byte global loads and stores on both sides, index math by shifts (the scalar form's 4-byte
// accesses and two runtime divisions per element ran it at ~0.7 TB/s)
__global__ void __launch_bounds__(256) conv_perm_tile4_k(const float* __restrict__ in, float* __restrict__ out,
                                                         int li, int lk, int inverse) {
  extern __shared__ float tile[];   // I * (K + 1)
  const int I = 1 << li, K = 1 << lk, K1 = K + 1;
  const int64_t base = (int64_t)blockIdx.x * I * K;
  const int n4 = (I * K) >> 2;
  const float4* in4 = reinterpret_cast<const float4*>(in + base);
  float4* out4 = reinterpret_cast<float4*>(out + base);
  if (!inverse) {   // in (i, k) -> out (k, i)
    for (int t = threadIdx.x; t < n4; t += 256) {
      const int e = t << 2, i = e >> lk, k = e & (K - 1);
      const float4 v = in4[t];
      float* d = tile + i * K1 + k;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n4; t += 256) {
      const int e = t << 2, k = e >> li, i = e & (I - 1);
      const float* sp = tile + i * K1 + k;
      out4[t] = make_float4(sp[0], sp[K1], sp[2 * K1], sp[3 * K1]);
    }
  } else {          // in (k, i) -> out (i, k)
    for (int t = threadIdx.x; t < n4; t += 256) {
      const int e = t << 2, k = e >> li, i = e & (I - 1);
      const float4 v = in4[t];
      float* d = tile + i * K1 + k;
      d[0] = v.x; d[K1] = v.y; d[2 * K1] = v.z; d[3 * K1] = v.w;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n4; t += 256) {
      const int e = t << 2, i = e >> lk, k = e & (K - 1);
      const float* sp = tile + i * K1 + k;
      out4[t] = make_float4(sp[0], sp[1], sp[2], sp[3]);
    }
  }
}

__global__ void conv_tflip_k(const float* __restrict__ w, float* __restrict__ out, int64_t G, int64_t Og,
                             int64_t I, int64_t K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= G * Og * I * K) return;
  // w layout: [(g*Og+o)][i][k]
  const int64_t k = idx % K, i = (idx / K) % I, o = (idx / (K * I)) % Og, g = idx / (K * I * Og);
  const int64_t kp = K - 1 - k;
  out[((g * I + i) * K + kp) * Og + o] = w[idx];
}

__global__ void wn_fwd_k(const float* __restrict__ g, const float* __restrict__ v, const float* __restrict__ sq,
                         float* __restrict__ w, float* __restrict__ norms, int64_t n, int64_t K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int64_t k = idx % K;
  const float nm = sqrtf(sq[k]);
  if (idx < K) norms[idx] = sqrtf(sq[idx]);
  w[idx] = g[k] * v[idx] / nm;
}

__global__ void wn_bwd_k(const float* __restrict__ g, const float* __restrict__ v, const float* __restrict__ norms,
                         const float* __restrict__ dw, const float* __restrict__ dwv, float* __restrict__ dg,
                         float* __restrict__ dv, int64_t n, int64_t K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  const int64_t k = idx % K;
  const float nm = norms[k];
  const float dgk = dwv[k] / nm;                 // sum(dw * v) / ||v||
  if (idx < K) dg[idx] = dwv[idx] / norms[idx];
  const float gk = g[k];
  // dv = (g/n) * (dw - (v/n) * dg)
  dv[idx] = gk / nm * (dw[idx] - v[idx] / nm * dgk);
}

inline unsigned nblocks(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }
}  // namespace

// =====================================================================================
extern "C" int64_t b2p_colsum_workspace(int64_t M, int64_t N) {
  return ((M + kColsumRows - 1) / kColsumRows) * N;
}

extern "C" int b2p_colsum(const float* X, int64_t M, int64_t N, int64_t ld, float* out, int accumulate,
                          float* partial, b2p_stream_t stream) {
  B2P_CHECK_ARG(X && out && partial, "colsum: NULL pointer");
  return colsum_impl(X, nullptr, 1, M, N, ld, 0, 0, out, accumulate, partial, (hipStream_t)stream);
}

extern "C" int b2p_colsum_batched(const float* X, const float* Y, int64_t batch, int64_t M, int64_t N,
                                  int64_t ld, int64_t bstride, int mode, float* out, int accumulate,
                                  float* partial, b2p_stream_t stream) {
  B2P_CHECK_ARG(X && out && partial, "colsum_batched: NULL pointer");
  B2P_CHECK_ARG(mode != 2 || Y, "colsum_batched: mode 2 needs Y");
  return colsum_impl(X, Y, batch, M, N, ld, bstride, mode, out, accumulate, partial, (hipStream_t)stream);
}

// ------------------------------------------------------------------ batch bookkeeping on the device
// The reference's own per-batch tensor ops on the step's path, one launch each instead of torch's 2-3
// elementwise launches (and the masked_fill copy):
//   out_lens = ((in_lens - k) / s).to(int32)   (src/model/b2p2t_model.py:170-173: int64 minus int, true
//              division in float32, truncation toward zero)
//   out_t    = where(t < 1, -100, t)            (src/model/w2v_custom_feat_extractor.py:70,
//              w2v_conformer_custom_feat_extractor.py:41)
__global__ void unfold_lens_k(const int64_t* __restrict__ in, int32_t* __restrict__ out, int64_t n, int64_t k, float s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)(__fdiv_rn((float)(in[i] - k), s));
}
__global__ void ctc_targets_k(const int64_t* __restrict__ t, int64_t* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t v = t[i];
    out[i] = v < 1 ? -100 : v;
  }
}

extern "C" int b2p_unfold_lens(const int64_t* in_lens, int32_t* out_lens, int64_t n, int64_t kernel, int64_t stride,
                               b2p_stream_t stream) {
  B2P_CHECK_ARG(in_lens && out_lens, "unfold_lens: NULL pointer");
  B2P_CHECK_ARG(stride > 0, "unfold_lens: stride must be positive");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(unfold_lens_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, in_lens, out_lens, n, kernel,
                     (float)stride);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_ctc_targets(const int64_t* targets, int64_t* out, int64_t n, b2p_stream_t stream) {
  B2P_CHECK_ARG(targets && out, "ctc_targets: NULL pointer");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ctc_targets_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, targets, out, n);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_scale_by_device_scalar(const float* x, const float* s, float* y, int64_t n, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && s && y, "scale_by_device_scalar: NULL pointer");
  B2P_CHECK_ARG(((uintptr_t)x & 15u) == 0 && ((uintptr_t)y & 15u) == 0, "scale_by_device_scalar: x / y 16-B aligned");
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int64_t n4 = n / 4;
  if (n4) hipLaunchKernelGGL(scale_dev_k, dim3(nblocks(n4)), dim3(256), 0, st, reinterpret_cast<const float4*>(x), s,
                             reinterpret_cast<float4*>(y), n4);
  if (n > 4 * n4) hipLaunchKernelGGL(scale_dev_tail_k, dim3(1), dim3(256), 0, st, x, s, y, 4 * n4, n);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "dropout: NULL pointer");
  B2P_CHECK_ARG(p >= 0.f && p < 1.f, "dropout: p must be in [0,1)");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dropout_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, x, y, n,
                     b2p_dropout_threshold(p), p > 0.f ? 1.f / (1.f - p) : 1.f, seed, b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layernorm_fwd16(const float* x, const float* gamma, const float* beta, float* y, uint16_t* y16,
                                   float* mean, float* rstd, int64_t rows, int64_t cols, float eps, float drop_p,
                                   uint64_t drop_seed, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && gamma && beta && y && mean && rstd, "layernorm_fwd: NULL pointer");
  B2P_CHECK_ARG(cols % 4 == 0 && cols <= 64 * 4 * LN_MAXV, "layernorm_fwd: cols must be %%4 and <= 1024");
  B2P_CHECK_ARG(((uintptr_t)y16 & 7u) == 0, "layernorm_fwd: y16 must be 8-byte aligned");
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(ln_fwd_k, dim3(nblocks(rows, 4)), dim3(256), 0, (hipStream_t)stream, x, gamma, beta, y,
                     mean, rstd, rows, (int)cols, eps, b2p_dropout_threshold(drop_p),
                     drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f, drop_seed, drop_p, y16, b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layernorm_fwd_x16(const float* x, const float* gamma, const float* beta, float* y, uint16_t* y16,
                                     int y16_fp16, uint16_t* y16b, float* mean, float* rstd, int64_t rows,
                                     int64_t cols, float eps, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && gamma && beta && y16 && mean && rstd, "layernorm_fwd_x16: NULL pointer");
  B2P_CHECK_ARG(cols % 4 == 0 && cols <= 64 * 4 * LN_MAXV, "layernorm_fwd_x16: cols must be %%4 and <= 1024");
  B2P_CHECK_ARG(((uintptr_t)y16 & 7u) == 0 && ((uintptr_t)y16b & 7u) == 0,
                "layernorm_fwd_x16: y16 / y16b must be 8-byte aligned");
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(ln_fwd_k, dim3(nblocks(rows, 4)), dim3(256), 0, (hipStream_t)stream, x, gamma, beta, y,
                     mean, rstd, rows, (int)cols, eps, 0u, 1.f, (uint64_t)0, 0.f, y16, b2p_seed_epoch(),
                     y16_fp16 ? 1 : 0, y16b);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layernorm_rotary16(const float* x, const float* gamma, const float* beta, float* mean, float* rstd,
                                      int64_t rows, int64_t cols, float eps, int64_t T, int64_t head_dim,
                                      const float* cos_t, const float* sin_t, int half16, uint16_t* h16,
                                      uint16_t* h16b, uint16_t* hr16, uint16_t* hr16b, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && gamma && beta && mean && rstd && cos_t && sin_t, "layernorm_rotary16: NULL pointer");
  B2P_CHECK_ARG(cols % 256 == 0 && cols <= 64 * 4 * LN_MAXV && cols % head_dim == 0,
                "layernorm_rotary16: cols must be a multiple of 256 (<= 1024) and of the head dim");
  B2P_CHECK_ARG(head_dim == 32 || head_dim == 64 || head_dim == 128 || head_dim == 256,
                "layernorm_rotary16: head dim must be 32, 64, 128 or 256");
  B2P_CHECK_ARG(T > 0 && rows % T == 0, "layernorm_rotary16: rows must be whole sequences of T");
  B2P_CHECK_ARG(((uintptr_t)x & 15u) == 0 && ((uintptr_t)cos_t & 15u) == 0 && ((uintptr_t)sin_t & 15u) == 0 &&
                    ((uintptr_t)h16 & 7u) == 0 && ((uintptr_t)h16b & 7u) == 0 && ((uintptr_t)hr16 & 7u) == 0 &&
                    ((uintptr_t)hr16b & 7u) == 0,
                "layernorm_rotary16: x / cos / sin 16-B and outputs 8-B aligned");
  if (rows <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(nblocks(rows, 4));
#define B2P_LNROT(HD)                                                                                            \
  hipLaunchKernelGGL(ln_rot16_k<HD>, grid, dim3(256), 0, st, x, gamma, beta, mean, rstd, rows, (int)cols, eps, \
                     (int)T, cos_t, sin_t, half16 ? 1 : 0, h16, h16b, hr16, hr16b)
  switch (head_dim) {
    case 32: B2P_LNROT(32); break;
    case 64: B2P_LNROT(64); break;
    case 128: B2P_LNROT(128); break;
    default: B2P_LNROT(256); break;
  }
#undef B2P_LNROT
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* mean,
                                 float* rstd, int64_t rows, int64_t cols, float eps, float drop_p,
                                 uint64_t drop_seed, b2p_stream_t stream) {
  return b2p_layernorm_fwd16(x, gamma, beta, y, nullptr, mean, rstd, rows, cols, eps, drop_p, drop_seed, stream);
}

namespace {
typedef void (*LnBwdKernel)(const float*, const float*, const float*, const float*, const float*, float*, const float*,
                            float*, int64_t, int, uint32_t, float, uint64_t, float, float*, uint32_t, float, uint64_t,
                            uint16_t*, const uint64_t*, const float*);
template <bool PF>
LnBwdKernel ln_bwd_pick(int mode) {
  switch (mode) {
    case 0: return ln_bwd_k<PF, 0>;
    case 1: return ln_bwd_k<PF, 1>;
    case 2: return ln_bwd_k<PF, 2>;
    case 3: return ln_bwd_k<PF, 3>;
    case 4: return ln_bwd_k<PF, 4>;
    case 5: return ln_bwd_k<PF, 5>;
    case 6: return ln_bwd_k<PF, 6>;
    default: return ln_bwd_k<PF, 7>;
  }
}
LnBwdKernel ln_bwd_kernel(bool pf, int mode) { return pf ? ln_bwd_pick<true>(mode) : ln_bwd_pick<false>(mode); }
}  // namespace

extern "C" int64_t b2p_layernorm_bwd_workspace(int64_t rows, int64_t cols) {
  const int64_t nblk = (rows + LN_BWD_ROWS - 1) / LN_BWD_ROWS;
  return nblk * 3 * cols + 3 * cols + ((nblk + kColsumRows - 1) / kColsumRows) * 3 * cols;
}

extern "C" int b2p_layernorm_bwd16(const float* dy, const float* x, const float* gamma, const float* mean,
                                   const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                                   int64_t cols, const float* dx_accum, float drop_p, uint64_t drop_seed,
                                   float* dx_dropped, float in_drop_p, uint64_t in_drop_seed, float* dbias_in,
                                   uint16_t* d16, float* workspace, b2p_stream_t stream) {
  return b2p_layernorm_bwd_acc2(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, rows, cols, dx_accum, nullptr, drop_p,
                                drop_seed, dx_dropped, in_drop_p, in_drop_seed, dbias_in, d16, workspace, stream);
}

extern "C" int b2p_layernorm_bwd_acc2(const float* dy, const float* x, const float* gamma, const float* mean,
                                      const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                                      int64_t cols, const float* dx_accum, const float* dx_accum2, float drop_p,
                                      uint64_t drop_seed, float* dx_dropped, float in_drop_p, uint64_t in_drop_seed,
                                      float* dbias_in, uint16_t* d16, float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(dy && x && gamma && mean && rstd && dx && workspace, "layernorm_bwd: NULL pointer");
  B2P_CHECK_ARG(cols % 4 == 0 && cols <= 64 * 4 * LN_MAXV, "layernorm_bwd: cols must be %%4 and <= 1024");
  B2P_CHECK_ARG(((uintptr_t)d16 & 7u) == 0, "layernorm_bwd: d16 must be 8-byte aligned");
  if (rows <= 0) return 0;
  const int nblk = (int)((rows + LN_BWD_ROWS - 1) / LN_BWD_ROWS);
  hipStream_t st = (hipStream_t)stream;
  static const bool pf = getenv("B2P_LN_PREFETCH") ? atoi(getenv("B2P_LN_PREFETCH")) != 0 : true;
  const int mode = (dx_accum ? LNB_A1 : 0) | (dx_accum2 ? LNB_A2 : 0) | (dx_dropped ? LNB_DXD : 0);
  hipLaunchKernelGGL(ln_bwd_kernel(pf, mode), dim3(nblk), dim3(256), 0, st, dy, x, gamma, mean, rstd, dx, dx_accum, workspace,
                     rows, (int)cols, b2p_dropout_threshold(drop_p), drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f,
                     drop_seed, drop_p, dx_dropped, b2p_dropout_threshold(in_drop_p),
                     in_drop_p > 0.f ? 1.f / (1.f - in_drop_p) : 1.f, in_drop_seed, d16, b2p_seed_epoch(), dx_accum2);
  // partials [nblk][3][cols] -> dgamma | dbeta | dbias_in in one launch
  B2P_CHECK_ARG(((uintptr_t)dgamma & 15u) == 0 && ((uintptr_t)dbeta & 15u) == 0 && ((uintptr_t)dbias_in & 15u) == 0,
                "layernorm_bwd: dgamma / dbeta / dbias_in must be 16-byte aligned");
  if (dgamma || dbeta || (dx_dropped && dbias_in))   // else the caller sums the partials later
    hipLaunchKernelGGL(ln_param_reduce_k, dim3((unsigned)((3 * cols + 127) / 128)), dim3(256), 0, st, workspace,
                       nblk, (int)cols, dgamma, dbeta, dx_dropped ? dbias_in : nullptr);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean,
                                 const float* rstd, float* dx, float* dgamma, float* dbeta, int64_t rows,
                                 int64_t cols, const float* dx_accum, float drop_p, uint64_t drop_seed,
                                 float* dx_dropped, float in_drop_p, uint64_t in_drop_seed, float* dbias_in,
                                 float* workspace, b2p_stream_t stream) {
  return b2p_layernorm_bwd16(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, rows, cols, dx_accum, drop_p, drop_seed,
                             dx_dropped, in_drop_p, in_drop_seed, dbias_in, nullptr, workspace, stream);
}

// ------------------------------------------------------------------ fp32 -> bf16 cast
__global__ void cast_bf16_k(const float* __restrict__ x, uint16_t* __restrict__ y, int64_t n4, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) {
    reinterpret_cast<uint2*>(y)[i] = b2p_pack_bf16x4(reinterpret_cast<const float4*>(x)[i]);
  } else if (i == n4) {
    for (int64_t j = 4 * n4; j < n; ++j) y[j] = b2p_bf16_bits(x[j]);
  }
}

extern "C" int b2p_cast_bf16(const float* x, uint16_t* y, int64_t n, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "cast_bf16: NULL pointer");
  B2P_CHECK_ARG(((uintptr_t)x & 15u) == 0 && ((uintptr_t)y & 7u) == 0, "cast_bf16: misaligned pointers");
  if (n <= 0) return 0;
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(cast_bf16_k, dim3(nblocks(n4 + 1)), dim3(256), 0, (hipStream_t)stream, x, y, n4, n);
  B2P_CHECK_LAUNCH();
  return 0;
}

// R x C block cast to bf16 / fp16: one thread per 4 columns of a row (16-B loads, 8-B stores when
// both strides and pointers allow, scalar otherwise)
template <bool H, bool VEC>
__global__ void __launch_bounds__(256) cast16_2d_k(const float* __restrict__ x, int64_t R, int64_t C, int64_t ldx,
                                                   uint16_t* __restrict__ y, int64_t ldy) {
  const int64_t c4 = (C + 3) / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * c4) return;
  const int64_t r = i / c4, c = (i - r * c4) * 4;
  const float* xs = x + r * ldx + c;
  uint16_t* ys = y + r * ldy + c;
  auto cvt = [](float v) -> uint16_t {
    if constexpr (H) return b2p_f16_bits(v);
    else return b2p_bf16_bits(v);
  };
  if (VEC && c + 4 <= C) {
    const float4 v = *reinterpret_cast<const float4*>(xs);
    *reinterpret_cast<uint2*>(ys) = make_uint2((uint32_t)cvt(v.x) | ((uint32_t)cvt(v.y) << 16),
                                               (uint32_t)cvt(v.z) | ((uint32_t)cvt(v.w) << 16));
  } else {
    for (int j = 0; j < 4 && c + j < C; ++j) ys[j] = cvt(xs[j]);
  }
}

extern "C" int b2p_cast16_2d(const float* x, int64_t R, int64_t C, int64_t ldx, uint16_t* y, int64_t ldy, int fp16,
                             b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "cast16_2d: NULL pointer");
  B2P_CHECK_ARG(R >= 0 && C >= 0 && ldx >= C && ldy >= C, "cast16_2d: bad shape / strides");
  if (R == 0 || C == 0) return 0;
  const bool vec = ((uintptr_t)x & 15u) == 0 && ((uintptr_t)y & 7u) == 0 && ldx % 4 == 0 && ldy % 4 == 0;
  const int64_t n = R * ((C + 3) / 4);
  const dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (fp16) {
    if (vec) hipLaunchKernelGGL((cast16_2d_k<true, true>), grid, dim3(256), 0, st, x, R, C, ldx, y, ldy);
    else hipLaunchKernelGGL((cast16_2d_k<true, false>), grid, dim3(256), 0, st, x, R, C, ldx, y, ldy);
  } else {
    if (vec) hipLaunchKernelGGL((cast16_2d_k<false, true>), grid, dim3(256), 0, st, x, R, C, ldx, y, ldy);
    else hipLaunchKernelGGL((cast16_2d_k<false, false>), grid, dim3(256), 0, st, x, R, C, ldx, y, ldy);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

// Split-bf16 operand of the bf16x3 mode: x (R x C fp32, ld ldx) = hi + lo with hi = bf16(x), lo =
// bf16(x - hi), written as three blocks (block b = lo when bit b of `pattern` is set, else hi), side by
// side in every row (along_cols: y[r][b*C + c], the k-contiguous operands) or stacked (y[b*R + r][c]).
// A GEMM over the 3x-deep K of an A image (hi, lo, hi) and a B image (hi, hi, lo) sums hi*hi + lo*hi +
// hi*lo in one launch on the bf16 MFMA kernels, with its full epilogue. pattern & 16: two blocks (the
// two-term images (hi, lo) . (hi, hi), one operand kept to ~16 bits, the other rounded to bf16).
__global__ void __launch_bounds__(256) split3_bf16_k(const float* __restrict__ x, int64_t R, int64_t C, int64_t ldx,
                                                     uint16_t* __restrict__ y, int64_t ldy, int pattern, int along_cols) {
  const int64_t c4 = (C + 3) / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= R * c4) return;
  const int64_t r = i / c4, c = (i - r * c4) * 4;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  const int nv = C - c < 4 ? (int)(C - c) : 4;
  const float* xs = x + r * ldx + c;
  if (nv == 4 && ((uintptr_t)xs & 15u) == 0) {
    const float4 q = *reinterpret_cast<const float4*>(xs);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {   // unrolled with guards: a runtime-bounded loop indexed the arrays in scratch memory
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < nv) v[j] = xs[j];
  }
  uint16_t hb[4], lb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 h = (__bf16)v[j];
    const __bf16 l = (__bf16)(v[j] - (float)h);
    hb[j] = __builtin_bit_cast(uint16_t, h);
    lb[j] = __builtin_bit_cast(uint16_t, l);
  }
  const uint2 hv = make_uint2((uint32_t)hb[0] | ((uint32_t)hb[1] << 16), (uint32_t)hb[2] | ((uint32_t)hb[3] << 16));
  const uint2 lv = make_uint2((uint32_t)lb[0] | ((uint32_t)lb[1] << 16), (uint32_t)lb[2] | ((uint32_t)lb[3] << 16));
  const int nb = (pattern & 16) ? 2 : 3;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    if (b >= nb) break;
    uint16_t* ys = along_cols ? y + r * ldy + b * C + c : y + (b * R + r) * ldy + c;
    const bool lo = (pattern >> b) & 1;
    if (nv == 4 && ((uintptr_t)ys & 7u) == 0) {
      *reinterpret_cast<uint2*>(ys) = lo ? lv : hv;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j < nv) ys[j] = lo ? lb[j] : hb[j];
    }
  }
}

extern "C" int b2p_split3_bf16(const float* x, int64_t R, int64_t C, int64_t ldx, uint16_t* y, int64_t ldy, int pattern,
                               int along_cols, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "split3_bf16: NULL pointer");
  B2P_CHECK_ARG(R >= 0 && C >= 0 && ldx >= C && ldy >= (along_cols ? ((pattern & 16) ? 2 : 3) * C : C),
                "split3_bf16: bad shape / strides");
  if (R == 0 || C == 0) return 0;
  const int64_t n = R * ((C + 3) / 4);
  hipLaunchKernelGGL(split3_bf16_k, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, R, C, ldx,
                     y, ldy, pattern, along_cols);
  B2P_CHECK_LAUNCH();
  return 0;
}

// y[c][r] = bf16(x[r][c]) for an R x C fp32 matrix written into columns col0 .. col0+R-1 of a
// [C][ldy] bf16 matrix (several row blocks stacked side by side: the transposed [Wq; Wk; Wv]):
// 64 x 64 tiles through LDS, reads and writes coalesced along the rows of x and y
__global__ void __launch_bounds__(256) transpose16_k(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                     int64_t R, int64_t C, int64_t ldy, int64_t col0) {
  __shared__ float tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? x[r * C + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < C && r < R) y[c * ldy + col0 + r] = b2p_bf16_bits(tile[tx][i]);
  }
}

extern "C" int b2p_transpose_bf16(const float* x, uint16_t* y, int64_t R, int64_t C, int64_t ldy, int64_t col0,
                                  b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "transpose_bf16: NULL pointer");
  B2P_CHECK_ARG(R >= 0 && C >= 0 && ldy >= col0 + R, "transpose_bf16: bad shape");
  if (R == 0 || C == 0) return 0;
  hipLaunchKernelGGL(transpose16_k, dim3((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64)), dim3(256), 0,
                     (hipStream_t)stream, x, y, R, C, ldy, col0);
  B2P_CHECK_LAUNCH();
  return 0;
}

// Unfold((k, 1), stride) of a (B, L, C) tensor, tap-major (feature tap*C + c), materialised as
// bf16 rows of k*C: row (b, t) is the contiguous slab x[b][t*stride .. t*stride+k)[.] cast to bf16
// (the GRU layer-0 weight-gradient GEMM operand; b2p2t_model.py:108-113,162-167).
__global__ void unfold16_k(const float* __restrict__ x, uint16_t* __restrict__ u, int64_t n4, int64_t L, int64_t C,
                           int64_t T, int64_t row4, int64_t stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int64_t row = i / row4, w = i - row * row4;
  const int64_t b = row / T, t = row - b * T;
  const float4 v = reinterpret_cast<const float4*>(x + (b * L + t * stride) * C)[w];
  reinterpret_cast<uint2*>(u)[i] = b2p_pack_bf16x4(v);
}

extern "C" int b2p_unfold16(const float* x, uint16_t* u, int64_t B, int64_t L, int64_t C, int64_t k, int64_t stride,
                            b2p_stream_t stream) {
  B2P_CHECK_ARG(x && u, "unfold16: NULL pointer");
  B2P_CHECK_ARG(C % 4 == 0 && ((uintptr_t)x & 15u) == 0 && ((uintptr_t)u & 7u) == 0, "unfold16: alignment");
  B2P_CHECK_ARG(L >= k && stride > 0, "unfold16: window longer than the sequence");
  const int64_t T = (L - k) / stride + 1;
  const int64_t n4 = B * T * k * C / 4;
  if (n4 <= 0) return 0;
  hipLaunchKernelGGL(unfold16_k, dim3(nblocks(n4)), dim3(256), 0, (hipStream_t)stream, x, u, n4, L, C, T, k * C / 4,
                     stride);
  B2P_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ implicit Unfold operands
// The Unfold((k,1), stride s) of a (B, L, C) tensor with L % s == 0 and k % s == 0 is never
// materialised: its row (b, t) is the contiguous slab x[b][s*t .. s*t+k)[.], i.e. row b*(L/s) + t of
// the flat tensor read with row stride s*C (overlapping rows). Three GEMMs use that view
// (functional._GRULayer): the layer-0 projection gi = U W^T, its weight gradient dW = dgi^T U, and
// the input gradient, computed without the (B*T, k*C) fp32 matrix and its col2im as
//   dX viewed (B*L/s, s*C) = G (B*L/s, (k/s)*N) . Wb ((k/s)*N, s*C),
//   G row (b, q) = dgi rows t = q-k/s+1 .. q of sample b (zero outside [0, T)),
//   Wb[j*N + n][r*C + c] = W[n][c*k + s*(k/s-1-j) + r].
// G is the overlapping-row view (row stride N) of dgi laid out with k/s-1 zero rows in front and
// L/s rows per sample (rows t >= T zero): b2p_pad_rows16 writes that layout.

// One workgroup per weight row n of W (reference layout [n][c*k + tap]): the row is transposed
// through LDS (row stride k+1: conflict-free tap-major reads); writes wf[n][tap*C + c] (16-bit,
// fp16 when half) and, when wb != NULL, the k/s rows wb[j*Ntot + n][.] (bf16).
__global__ void __launch_bounds__(256) unfold_weight16_k(const float* __restrict__ w0, const float* __restrict__ w1,
                                                         int64_t G, int C, int k, int s, uint16_t* __restrict__ wf,
                                                         int half, uint16_t* __restrict__ wb, int64_t Ntot) {
  extern __shared__ float tile[];   // C * (k + 1)
  const int64_t n = blockIdx.x;
  const int CK = C * k;
  const float* src = n < G ? w0 + n * CK : w1 + (n - G) * CK;
  for (int t = threadIdx.x; t < CK; t += 256) {
    const int c = t / k, tap = t - c * k;
    tile[c * (k + 1) + tap] = src[t];
  }
  __syncthreads();
  const int C4 = C / 4;
  for (int e4 = threadIdx.x; e4 < CK / 4; e4 += 256) {   // 4 consecutive channels of one tap
    const int tap = e4 / C4, c = 4 * (e4 - tap * C4);
    const float* tp = tile + c * (k + 1) + tap;
    const float4 v = make_float4(tp[0], tp[k + 1], tp[2 * (k + 1)], tp[3 * (k + 1)]);
    reinterpret_cast<uint2*>(wf + n * CK)[e4] = b2p_pack16x4(v, half != 0);
  }
  if (!wb) return;
  const int J = k / s, SC = s * C;
  for (int e4 = threadIdx.x; e4 < CK / 4; e4 += 256) {
    const int e = 4 * e4;
    const int j = e / SC, rc = e - j * SC;
    const int r = rc / C, c = rc - r * C;
    const int tap = s * (J - 1 - j) + r;
    const float* tp = tile + c * (k + 1) + tap;
    const float4 v = make_float4(tp[0], tp[k + 1], tp[2 * (k + 1)], tp[3 * (k + 1)]);
    *reinterpret_cast<uint2*>(wb + ((int64_t)j * Ntot + n) * SC + rc) = b2p_pack_bf16x4(v);
  }
}

extern "C" int b2p_unfold_weight16(const float* w0, const float* w1, int64_t G, int64_t C, int64_t k, int64_t stride,
                                   uint16_t* wf, int fp16, uint16_t* wb, b2p_stream_t stream) {
  B2P_CHECK_ARG(w0 && wf, "unfold_weight16: NULL pointer");
  B2P_CHECK_ARG(C % 4 == 0 && k > 0 && stride > 0 && k % stride == 0, "unfold_weight16: bad geometry");
  B2P_CHECK_ARG(((uintptr_t)wf & 7u) == 0 && ((uintptr_t)wb & 7u) == 0, "unfold_weight16: alignment");
  const size_t lds = (size_t)C * (k + 1) * sizeof(float);
  B2P_CHECK_ARG(lds <= 64 * 1024, "unfold_weight16: C * (k + 1) floats must fit 64 KB of LDS");
  const int64_t Ntot = w1 ? 2 * G : G;
  if (G <= 0) return 0;
  hipLaunchKernelGGL(unfold_weight16_k, dim3((unsigned)Ntot), dim3(256), lds, (hipStream_t)stream, w0, w1, G, (int)C,
                     (int)k, (int)stride, wf, fp16, wb, Ntot);
  B2P_CHECK_LAUNCH();
  return 0;
}

// dst row (lead + b*R + t) = bf16(src[b][t]) for t < T, every other row (the lead rows, t >= T) zero
__global__ void pad_rows16_k(const float* __restrict__ src, uint16_t* __restrict__ dst, int64_t T, int64_t R,
                             int64_t lead, int64_t N4, int64_t total4) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const int64_t row = i / N4, c4 = i - row * N4;
  uint2 v = make_uint2(0u, 0u);
  if (row >= lead) {
    const int64_t rr = row - lead, b = rr / R, t = rr - b * R;
    if (t < T) v = b2p_pack_bf16x4(reinterpret_cast<const float4*>(src + (b * T + t) * N4 * 4)[c4]);
  }
  reinterpret_cast<uint2*>(dst)[i] = v;
}

extern "C" int b2p_pad_rows16(const float* src, uint16_t* dst, int64_t B, int64_t T, int64_t N, int64_t R,
                              int64_t lead, b2p_stream_t stream) {
  B2P_CHECK_ARG(src && dst, "pad_rows16: NULL pointer");
  B2P_CHECK_ARG(N % 4 == 0 && R >= T && lead >= 0, "pad_rows16: bad geometry");
  B2P_CHECK_ARG(((uintptr_t)src & 15u) == 0 && ((uintptr_t)dst & 7u) == 0, "pad_rows16: alignment");
  const int64_t total4 = (lead + B * R) * (N / 4);
  if (total4 <= 0) return 0;
  hipLaunchKernelGGL(pad_rows16_k, dim3(nblocks(total4)), dim3(256), 0, (hipStream_t)stream, src, dst, T, R, lead,
                     N / 4, total4);
  B2P_CHECK_LAUNCH();
  return 0;
}

// y[i] = 16-bit(x[i]) for i < n, 0 for n <= i < n_total (the zero tail an overlapping-row view reads)
__global__ void cast16_tail_k(const float* __restrict__ x, uint16_t* __restrict__ y, int64_t n4, int64_t total4,
                              int half) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  reinterpret_cast<uint2*>(y)[i] = i < n4 ? b2p_pack16x4(reinterpret_cast<const float4*>(x)[i], half != 0)
                                          : make_uint2(0u, 0u);
}

extern "C" int b2p_cast16_tail(const float* x, uint16_t* y, int64_t n, int64_t n_total, int fp16,
                               b2p_stream_t stream) {
  B2P_CHECK_ARG(x && y, "cast16_tail: NULL pointer");
  B2P_CHECK_ARG(n % 4 == 0 && n_total % 4 == 0 && n_total >= n, "cast16_tail: sizes must be multiples of 4");
  B2P_CHECK_ARG(((uintptr_t)x & 15u) == 0 && ((uintptr_t)y & 7u) == 0, "cast16_tail: alignment");
  if (n_total <= 0) return 0;
  hipLaunchKernelGGL(cast16_tail_k, dim3(nblocks(n_total / 4)), dim3(256), 0, (hipStream_t)stream, x, y, n / 4,
                     n_total / 4, fp16);
  B2P_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ small-tensor assembly
// dst = (a ? a : 0) + (b ? b : 0) over `count` floats, up to GATHER_MAXR records per launch (one
// grid row each): the per-step stacking / concatenation of GRU weights and biases (W_hh of both
// directions, folded b_ih + b_hh[r,z]) in one launch instead of a torch cat / stack / add each.
constexpr int GATHER_MAXR = 16;
struct GatherRecs { int64_t r[GATHER_MAXR][4]; };
__global__ void gather_rec_k(GatherRecs g) {
  const int64_t* r = g.r[blockIdx.y];
  float* dst = reinterpret_cast<float*>(r[0]);
  const float* a = reinterpret_cast<const float*>(r[1]);
  const float* b = reinterpret_cast<const float*>(r[2]);
  const int64_t n = r[3];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (a ? a[i] : 0.f) + (b ? b[i] : 0.f);
}

extern "C" int b2p_gather_recs(const int64_t* recs, int nrec, b2p_stream_t stream) {
  B2P_CHECK_ARG(recs != nullptr || nrec == 0, "gather_recs: NULL records");
  for (int c0 = 0; c0 < nrec; c0 += GATHER_MAXR) {
    const int nc = nrec - c0 < GATHER_MAXR ? nrec - c0 : GATHER_MAXR;
    GatherRecs g;
    int64_t maxn = 0;
    for (int i = 0; i < nc; ++i) {
      for (int k = 0; k < 4; ++k) g.r[i][k] = recs[4 * (c0 + i) + k];
      B2P_CHECK_ARG(g.r[i][3] <= 0 || g.r[i][0], "gather_recs: NULL destination");
      maxn = g.r[i][3] > maxn ? g.r[i][3] : maxn;
    }
    if (maxn <= 0) continue;
    const int64_t bx = (maxn + 255) / 256;
    hipLaunchKernelGGL(gather_rec_k, dim3((unsigned)(bx < 512 ? bx : 512), (unsigned)nc), dim3(256), 0,
                       (hipStream_t)stream, g);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_softmax_fwd(const float* S, float* P, float* Pd, int64_t rows, int64_t n, int64_t ld,
                               float drop_p, uint64_t drop_seed, b2p_stream_t stream) {
  B2P_CHECK_ARG(S && P && Pd, "softmax_fwd: NULL pointer");
  B2P_CHECK_ARG(n > 0 && n <= 64 * SM_MAXE && ld >= n && ld <= 64 * SM_MAXE, "softmax_fwd: row length must be <= 512");
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(softmax_fwd_k, dim3(nblocks(rows, 4)), dim3(256), 0, (hipStream_t)stream, S, P, Pd, rows,
                     (int)n, ld, b2p_dropout_threshold(drop_p), drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f,
                     drop_seed, drop_p, b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_softmax_bwd(const float* P, const float* dPd, float* dS, int64_t rows, int64_t n, int64_t ld,
                               float drop_p, uint64_t drop_seed, b2p_stream_t stream) {
  B2P_CHECK_ARG(P && dPd && dS, "softmax_bwd: NULL pointer");
  B2P_CHECK_ARG(n > 0 && n <= 64 * SM_MAXE && ld >= n && ld <= 64 * SM_MAXE, "softmax_bwd: row length must be <= 512");
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(softmax_bwd_k, dim3(nblocks(rows, 4)), dim3(256), 0, (hipStream_t)stream, P, dPd, dS, rows,
                     (int)n, ld, b2p_dropout_threshold(drop_p), drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f,
                     drop_seed, drop_p, b2p_seed_epoch());
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_act_bwd(const float* dy, const float* pre, float* dx, int64_t n, int act, b2p_stream_t stream) {
  B2P_CHECK_ARG(dy && pre && dx, "act_bwd: NULL pointer");
  if (n <= 0) return 0;
  if (n % 4 == 0 && (((uintptr_t)dy | (uintptr_t)pre | (uintptr_t)dx) & 15u) == 0)
    hipLaunchKernelGGL(act_bwd4_k, dim3(nblocks(n / 4)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(dy), reinterpret_cast<const float4*>(pre),
                       reinterpret_cast<float4*>(dx), n / 4, act);
  else
    hipLaunchKernelGGL(act_bwd_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, dy, pre, dx, n, act);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_gauss_smooth(const float* x, const float* taps, int ntaps, float* y, int64_t B, int64_t L,
                                int64_t C, b2p_stream_t stream) {
  B2P_CHECK_ARG(x && taps && y, "gauss_smooth: NULL pointer");
  B2P_CHECK_ARG(C % 4 == 0 && ntaps > 0, "gauss_smooth: C must be %%4");
  const int64_t n = B * L * (C / 4);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gauss_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, x, taps, ntaps, y, B, L, C / 4);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_unfold_col2im(const float* dA, const float* Z, float* dX, int64_t B, int64_t L, int64_t C,
                                 int64_t T, int ktaps, int stride, b2p_stream_t stream) {
  B2P_CHECK_ARG(dA && dX, "unfold_col2im: NULL pointer");
  B2P_CHECK_ARG(C % 4 == 0 && stride > 0 && ktaps > 0, "unfold_col2im: bad geometry");
  const int64_t n = B * L * (C / 4);
  if (n <= 0) return 0;
  hipLaunchKernelGGL(col2im_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, dA, Z, dX, B, L, C / 4, T,
                     ktaps, stride);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_day_reduce(const float* per_sample, const int64_t* day_idx, int64_t B, int64_t ndays,
                              int64_t elems, float* out, b2p_stream_t stream) {
  B2P_CHECK_ARG(per_sample && day_idx && out, "day_reduce: NULL pointer");
  const int64_t n = ndays * elems;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(day_reduce_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, per_sample, day_idx, B,
                     ndays, elems, out);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_conv_weight_permute(const float* in, float* out, int64_t O, int64_t I, int64_t ntaps,
                                       int inverse, b2p_stream_t stream) {
  B2P_CHECK_ARG(in && out && in != out, "conv_weight_permute: bad pointers");
  const int64_t n = O * I * ntaps;
  if (n <= 0) return 0;
  const size_t lds = (size_t)I * (ntaps + 1) * sizeof(float);
  auto pow2 = [](int64_t v) { return v >= 4 && (v & (v - 1)) == 0; };
  if (lds <= 64 * 1024 && O < (1ll << 31) && pow2(I) && pow2(ntaps) && ((uintptr_t)in & 15u) == 0 &&
      ((uintptr_t)out & 15u) == 0)
    hipLaunchKernelGGL(conv_perm_tile4_k, dim3((unsigned)O), dim3(256), lds, (hipStream_t)stream, in, out,
                       __builtin_ctzll((unsigned long long)I), __builtin_ctzll((unsigned long long)ntaps), inverse);
  else if (lds <= 64 * 1024 && O < (1ll << 31))
    hipLaunchKernelGGL(conv_perm_tile_k, dim3((unsigned)O), dim3(256), lds, (hipStream_t)stream, in, out, (int)I,
                       (int)ntaps, inverse);
  else
    hipLaunchKernelGGL(conv_perm_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, in, out, O, I, ntaps,
                       inverse);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_conv_weight_transpose_flip(const float* w, float* out, int64_t G, int64_t Og, int64_t I,
                                              int64_t ntaps, b2p_stream_t stream) {
  B2P_CHECK_ARG(w && out && w != out, "conv_weight_transpose_flip: bad pointers");
  const int64_t n = G * Og * I * ntaps;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(conv_tflip_k, dim3(nblocks(n)), dim3(256), 0, (hipStream_t)stream, w, out, G, Og, I, ntaps);
  B2P_CHECK_LAUNCH();
  return 0;
}

// workspace: K floats (sum of squares) + colsum partials
extern "C" int64_t b2p_weight_norm_workspace(int64_t O, int64_t I, int64_t K) {
  return K + b2p_colsum_workspace(O * I, K);
}

extern "C" int b2p_weight_norm_fwd(const float* g, const float* v, float* w, float* norms, int64_t O, int64_t I,
                                   int64_t K, float* workspace, b2p_stream_t stream) {
  B2P_CHECK_ARG(g && v && w && norms && workspace, "weight_norm_fwd: NULL pointer");
  hipStream_t st = (hipStream_t)stream;
  float* sq = workspace;
  if (colsum_impl(v, nullptr, 1, O * I, K, K, 0, 1, sq, 0, workspace + K, st)) return 1;
  const int64_t n = O * I * K;
  hipLaunchKernelGGL(wn_fwd_k, dim3(nblocks(n)), dim3(256), 0, st, g, v, sq, w, norms, n, K);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_weight_norm_bwd(const float* g, const float* v, const float* norms, const float* dw, float* dg,
                                   float* dv, int64_t O, int64_t I, int64_t K, float* workspace,
                                   b2p_stream_t stream) {
  B2P_CHECK_ARG(g && v && norms && dw && dg && dv && workspace, "weight_norm_bwd: NULL pointer");
  hipStream_t st = (hipStream_t)stream;
  float* dwv = workspace;
  if (colsum_impl(dw, v, 1, O * I, K, K, 0, 2, dwv, 0, workspace + K, st)) return 1;
  const int64_t n = O * I * K;
  hipLaunchKernelGGL(wn_bwd_k, dim3(nblocks(n)), dim3(256), 0, st, g, v, norms, dw, dwv, dg, dv, n, K);
  B2P_CHECK_LAUNCH();
  return 0;
}
