// Plain 16-bit GEMMs through hipBLASLt (the vendor library), everything else on the hand-written kernels.
//
// "Plain" = a GEMM whose epilogue is only alpha / beta / an added matrix: D = alpha * A B^T (+ beta * C or
// + residual R), written as fp32 or as one 16-bit copy, one batch member, dense operands (no implicit conv
// view, no gathered batch, leading dimensions >= the contiguous extent). In the training step these are the
// backward-data GEMMs: dO = dZ Wo (16-bit output), the QKV / FFN1 / pointwise-conv input gradients with
// the block's residual gradient added, the GRU / front-end input gradients. Every fused GEMM (bias,
// activation, dropout, act', 16-bit copies beside fp32, column sums, split-bf16 images, LayerDrop-gated
// forward work, batched weight gradients) stays on gemm16 / gemm16_pp (gemm16.hip), which the yardstick
// (profiles/r05c_gemm_vs_blas.txt) measured at or ahead of hipBLASLt on the weight-gradient shapes and
// which carry the epilogues the library does not have.
//
// LayerDrop: a plain GEMM of a layer this replay skips runs anyway (the library cannot read the device
// gate). Its A operand is then an exact-zero gradient (the skipped layer's incoming gradient is zero-filled
// by ld_route_k and every gradient inside the layer is linear in it), so D equals what the gated kernel
// writes (acc = 0, then beta C / residual): same values, only the dropped work is not saved.
//
// Plans (matmul descriptor, layouts, the heuristic's first algorithm) are cached per shape key and made
// only outside stream capture (the eager first step of every shape makes them); a capture that meets an
// unplanned shape uses the hand-written kernel. No workspace: algorithms that need one are not offered
// (HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES = 0), which also excludes the stream-K forms whose
// fix-up order could vary between runs. B2P_BLASLT=0 disables the path.
//
// Layout: our matrices are row-major; hipBLASLt is column-major. Row-major C (M x N, ldc) is the
// column-major (N x M, ldc) matrix C^T = B A^T, so the library's "A" is our B and its "B" is our A:
//   our B k-contiguous ([n][k], ldb): column-major (K x N, ldb) = B^T -> op T;  n-contiguous ([k][n]):
//   column-major (N x K, ldb) = B -> op N.  Our A k-contiguous ([m][k], lda): column-major (K x M) = A^T
//   -> op N;  m-contiguous ([k][m]): column-major (M x K) = A -> op T.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "common.h"
#include "../../include/b2p_hip.h"

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo;
  bool ok = false;
};

// (M, N, K, AK, BK, lda, ldb, ldc_in, ldd, in type, out type, has C)
typedef std::tuple<int64_t, int64_t, int64_t, int, int, int64_t, int64_t, int64_t, int64_t, int, int, int> Key;

std::mutex g_mu;
hipblasLtHandle_t g_handle = nullptr;
int g_enabled = -1;            // -1: not decided yet
std::map<Key, Plan> g_plans;
long long g_calls = 0;         // launches that went to the library (tests / diagnostics)
// B2P_BLASLT_WS=<MiB>: offer the heuristic algorithms that need a workspace (one buffer, allocated once
// outside capture; measurement switch: the default 0 keeps the deterministic no-workspace forms)
void* g_ws = nullptr;
uint64_t g_ws_bytes = 0;
int g_ws_init = 0;

void ws_init() {
  if (g_ws_init) return;
  g_ws_init = 1;
  const char* e = getenv("B2P_BLASLT_WS");
  const uint64_t mb = e ? strtoull(e, nullptr, 10) : 0;
  if (mb && hipMalloc(&g_ws, mb << 20) == hipSuccess) g_ws_bytes = mb << 20;
}

bool enabled() {
  if (g_enabled < 0) {
    const char* e = getenv("B2P_BLASLT");
    g_enabled = (e && e[0] == '0') ? 0 : 1;
  }
  return g_enabled == 1;
}

bool capturing(hipStream_t st) {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &s) != hipSuccess) return true;   // unknown: behave as in a capture
  return s != hipStreamCaptureStatusNone;
}

hipDataType in_type(const b2p_operand& o) { return o.dtype == 2 ? HIP_R_16F : HIP_R_16BF; }

// the shape and epilogue this path takes; out: 0 = fp32 C, 1 = 16-bit C16
bool eligible(const b2p_gemm_desc& d, int* out16) {
  const b2p_epilogue& e = d.ep;
  if (d.A.dtype == 0 || d.A.dtype != d.B.dtype) return false;
  if (d.A.conv || d.B.conv || d.A.gather1 || d.B.gather1) return false;
  if ((int64_t)d.nz1 * d.nz2 != 1) return false;
  // weight gradients (A m-contiguous: K = tokens) stay on gemm16_pp, measured ahead of the library there
  if (!d.A.inner_is_k) return false;
  if (e.bias || e.pre_out || e.act || e.act_bwd || e.drop_p != 0.f || e.pre16 || e.aux16 || e.colsum_part || e.C16b ||
      e.bias_gather)
    return false;
  if (b2p_gate_batch()) return false;
  const bool c32 = e.C != nullptr, c16 = e.C16 != nullptr;
  if (c32 == c16) return false;                                 // exactly one output
  if (c16 && (e.beta != 0.f || e.residual)) return false;       // the 16-bit output is a plain product
  if (e.residual && e.beta != 0.f) return false;                // residual or beta, not both
  // leading dimensions the library accepts (>= the contiguous extent): an overlapping-row view is ours
  if (d.A.inner_is_k ? d.A.ld < d.K : d.A.ld < d.M) return false;
  if (d.B.inner_is_k ? d.B.ld < d.K : d.B.ld < d.N) return false;
  if (e.ldc < d.N || (e.residual && e.ldr < d.N)) return false;
  if (d.M < 64 || d.N < 64 || d.K < 64) return false;           // tiny GEMMs: launch overhead dominates
  *out16 = c16 ? 1 : 0;
  return true;
}

bool make_plan(const b2p_gemm_desc& d, int out16, Plan& p) {
  const hipDataType ti = in_type(d.A);
  const hipDataType to = out16 ? ((d.ep.flags & B2P_EPI_C16_FP16) ? HIP_R_16F : HIP_R_16BF) : HIP_R_32F;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
  const int32_t ta = d.B.inner_is_k ? HIPBLAS_OP_T : HIPBLAS_OP_N;   // library A = our B
  const int32_t tb = d.A.inner_is_k ? HIPBLAS_OP_N : HIPBLAS_OP_T;   // library B = our A
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  // stored (rows, cols) of each column-major operand
  const uint64_t ar = d.B.inner_is_k ? d.K : d.N, ac = d.B.inner_is_k ? d.N : d.K;
  const uint64_t br = d.A.inner_is_k ? d.K : d.M, bc = d.A.inner_is_k ? d.M : d.K;
  const int64_t ldcin = d.ep.residual ? d.ep.ldr : d.ep.ldc;
  if (hipblasLtMatrixLayoutCreate(&p.la, ti, ar, ac, d.B.ld) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lb, ti, br, bc, d.A.ld) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.lc, to, d.N, d.M, ldcin) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatrixLayoutCreate(&p.ld, to, d.N, d.M, d.ep.ldc) != HIPBLAS_STATUS_SUCCESS)
    return false;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
  ws_init();
  const uint64_t ws = g_ws_bytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t s =
      hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.la, p.lb, p.lc, p.ld, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (s != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS || res[0].workspaceSize > ws)
    return false;
  p.algo = res[0].algo;
  p.ok = true;
  return true;
}

}  // namespace

// 1: launched through hipBLASLt; 0: not taken (the caller launches its own kernel); -1: a library error
int b2p_blaslt_gemm(const b2p_gemm_desc& d, hipStream_t st) {
  int out16 = 0;
  if (!enabled() || !eligible(d, &out16)) return 0;
  const int64_t ldcin = d.ep.residual ? d.ep.ldr : d.ep.ldc;
  const Key key(d.M, d.N, d.K, d.A.inner_is_k, d.B.inner_is_k, d.A.ld, d.B.ld, ldcin, d.ep.ldc, (int)d.A.dtype,
                out16 ? ((d.ep.flags & B2P_EPI_C16_FP16) ? 2 : 1) : 0, (d.ep.residual || d.ep.beta != 0.f) ? 1 : 0);
  Plan* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      if (capturing(st)) return 0;   // plans are made in eager launches only
      if (!g_handle && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) {
        g_enabled = 0;
        return 0;
      }
      Plan np;
      make_plan(d, out16, np);   // a shape the library does not plan stays on our kernel (ok = false)
      it = g_plans.emplace(key, np).first;
    }
    p = &it->second;
  }
  if (!p->ok) return 0;
  const float alpha = d.ep.alpha;
  const float beta = d.ep.residual ? 1.f : d.ep.beta;
  const void* C = d.ep.residual ? (const void*)d.ep.residual : (out16 ? (const void*)d.ep.C16 : (const void*)d.ep.C);
  void* D = out16 ? (void*)d.ep.C16 : (void*)d.ep.C;
  const hipblasStatus_t s = hipblasLtMatmul(g_handle, p->desc, &alpha, d.B.ptr, p->la, d.A.ptr, p->lb, &beta, C, p->lc,
                                            D, p->ld, &p->algo, g_ws, g_ws_bytes, st);
  if (s != HIPBLAS_STATUS_SUCCESS) {
    b2p_set_error("gemm: hipblasLtMatmul failed (status %d)", (int)s);
    return -1;
  }
  ++g_calls;
  return 1;
}

extern "C" int64_t b2p_blaslt_calls(int reset) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int64_t c = g_calls;
  if (reset) g_calls = 0;
  return c;
}

extern "C" int b2p_blaslt_enable(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_enabled = on ? 1 : 0;
  return 0;
}
