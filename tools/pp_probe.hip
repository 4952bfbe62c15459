// Diagnostic: per-workgroup clock stamps of the 256x256 ping-pong GEMM (start, after the prologue,
// after the K loop, end). Build: hipcc -O3 --offload-arch=gfx950 -DB2P_PP_STAMPS tools/pp_probe.hip
//   -Lwav2vec2forbrain_amd -lb2p_hip -o probe_bin/pp_probe ; run: probe_bin/pp_probe M N K
#define B2P_PP_STAMPS 1
#include "../wav2vec2forbrain_amd/csrc/gemm16.hip"
#include "../wav2vec2forbrain_amd/csrc/gemm16_nt.hip"
#include "../wav2vec2forbrain_amd/csrc/gemm16_nt16.hip"
#include "../wav2vec2forbrain_amd/csrc/gemm16_misc.hip"
#include <algorithm>
#include <vector>

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 2048, K = argc > 3 ? atoi(argv[3]) : 256;
  const int c16 = argc > 4 ? atoi(argv[4]) : 0;   // 0: fp32 C, 1: bf16 C16 only, 2: both + bias
  const int act = argc > 5 ? atoi(argv[5]) : 0;   // B2P_ACT_* in the epilogue
  const int tn = argc > 6 ? atoi(argv[6]) : 0;    // 1: both operands m/n-contiguous (the weight-gradient layout)
  std::vector<uint16_t> ha((size_t)M * K), hb((size_t)N * K);
  uint32_t x = 1;
  for (auto& v : ha) { x = x * 1664525u + 1013904223u; v = 0x3c00 + ((x >> 16) & 0x7f) + ((x >> 31) << 15); }
  for (auto& v : hb) { x = x * 1664525u + 1013904223u; v = 0x3c00 + ((x >> 16) & 0x7f) + ((x >> 31) << 15); }
  void *a, *b, *c;
  hipMalloc(&a, ha.size() * 2); hipMalloc(&b, hb.size() * 2); hipMalloc(&c, (size_t)M * N * 4);
  hipMemcpy(a, ha.data(), ha.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(b, hb.data(), hb.size() * 2, hipMemcpyHostToDevice);
  b2p_gemm_desc d{};
  d.M = M; d.N = N; d.K = K; d.nz1 = d.nz2 = 1;
  d.A.ptr = a; d.A.ld = tn ? M : K; d.A.inner_is_k = tn ? 0 : 1; d.A.dtype = 1;
  d.B.ptr = b; d.B.ld = tn ? N : K; d.B.inner_is_k = tn ? 0 : 1; d.B.dtype = 1;
  void *c2 = nullptr, *bias = nullptr;
  if (c16 == 1) d.ep.C16 = (uint16_t*)c;
  else d.ep.C = (float*)c;
  if (c16 == 2) {
    hipMalloc(&c2, (size_t)M * N * 2);
    hipMalloc(&bias, (size_t)N * 4);
    hipMemset(bias, 0, (size_t)N * 4);
    d.ep.C16 = (uint16_t*)c2;
    d.ep.bias = (const float*)bias;
  }
  d.ep.act = act;
  d.ep.ldc = N; d.ep.alpha = 1.f;
  if (getenv("PP_DIAG")) {   // K-loop ablation (gemm16_impl.inc g_pp_diag)
    const int dg = atoi(getenv("PP_DIAG"));
    hipMemcpyToSymbol(HIP_SYMBOL(g_pp_diag), &dg, sizeof(dg));
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int it = 0; it < 5; ++it) b2p_gemm16_launch(d, 0);
  hipEventRecord(e0, 0);
  const int iters = 20;
  for (int it = 0; it < iters; ++it) b2p_gemm16_launch(d, 0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const int nwg = ((M + 255) / 256) * ((N + 255) / 256);
  std::vector<unsigned long long> st((size_t)8 * 8192);
  hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_pp_stamps), st.size() * 8);
  printf("M %d N %d K %d  %s act %d: %.1f us/launch (%.1f TF/s), %d workgroups\n", M, N, K,
         c16 == 0 ? "C32" : c16 == 1 ? "C16" : "C32+C16+bias", act,
         1e3 * ms / iters, 2.0 * M * N * K / (ms / iters) / 1e9, nwg);
  if (getenv("B2P_GEMM16_PP") && atoi(getenv("B2P_GEMM16_PP")) == 0) return 0;
  // last launch's stamps
  unsigned long long r0 = ~0ull, r3 = 0;
  std::vector<double> pro, loop, epi, tot, startoff, endoff;
  for (int w = 0; w < std::min(nwg, 8192); ++w) {
    const unsigned long long* s = &st[(size_t)w * 8];
    r0 = std::min(r0, s[4]); r3 = std::max(r3, s[7]);
    pro.push_back((double)(s[1] - s[0])); loop.push_back((double)(s[2] - s[1])); epi.push_back((double)(s[3] - s[2]));
    tot.push_back((double)(s[3] - s[0]));
  }
  for (int w = 0; w < std::min(nwg, 8192); ++w) {
    const unsigned long long* s = &st[(size_t)w * 8];
    startoff.push_back((s[4] - r0) / 100.0); endoff.push_back((s[7] - r0) / 100.0);
  }
  auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
  printf("cycles (shader clock)  median / p90 / max:\n");
  printf("  prologue %8.0f %8.0f %8.0f\n", q(pro, .5), q(pro, .9), q(pro, 1));
  printf("  k-loop   %8.0f %8.0f %8.0f\n", q(loop, .5), q(loop, .9), q(loop, 1));
  printf("  epilogue %8.0f %8.0f %8.0f\n", q(epi, .5), q(epi, .9), q(epi, 1));
  printf("  total    %8.0f %8.0f %8.0f\n", q(tot, .5), q(tot, .9), q(tot, 1));
  printf("wall (us from first start): start median %.2f max %.2f; end median %.2f max %.2f\n", q(startoff, .5),
         q(startoff, 1), q(endoff, .5), q(endoff, 1));
  const double clk = q(tot, .5) / ((q(endoff, .5) - q(startoff, .5)) * 1e3);
  printf("in-kernel clock ~ %.2f GHz\n", clk);
  return 0;
}
