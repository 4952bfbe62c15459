// Diagnostic: ablations of the one-CU GRU forward recurrence (gru16_fwd<256, DIAG, SPLIT>): time per launch at
// the base step's shape (B 32, T' 249, H 256, 2 directions) with parts of the time step removed.
// Build: hipcc -O3 --offload-arch=gfx950 tools/gru_probe.hip -o probe_bin/gru_probe ; run: probe_bin/gru_probe [B T]
#include "../wav2vec2forbrain_amd/csrc/gru16.hip"
#include <cstdio>
#include <cstring>
#include <vector>

template <int DIAG, bool SPLIT = false>
static float time_fwd(const float* gi, const float* whh, const float* bhh, float* hL, float* sv, int B, int T, int nd) {
  const size_t shm = fwd_lds_bytes<256>();
  hipFuncSetAttribute((const void*)gru16_fwd<256, DIAG, SPLIT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  dim3 grid((unsigned)((B + BG - 1) / BG), (unsigned)nd);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 2; ++i)
    hipLaunchKernelGGL((gru16_fwd<256, DIAG, SPLIT>), grid, dim3(512), shm, 0, gi, whh, bhh, nullptr, hL, sv, B, T, nd);
  hipEventRecord(e0, 0);
  const int it = 5;
  for (int i = 0; i < it; ++i)
    hipLaunchKernelGGL((gru16_fwd<256, DIAG, SPLIT>), grid, dim3(512), shm, 0, gi, whh, bhh, nullptr, hL, sv, B, T, nd);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / it;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, T = argc > 2 ? atoi(argv[2]) : 249, H = 256, nd = 2;
  const size_t n1 = (size_t)b2p_gru16_lane_floats(B, T, H, nd, 1);
  std::vector<float> hgi(3 * n1), hw((size_t)nd * 3 * H * H), hb((size_t)nd * 3 * H);
  uint32_t x = 1;
  auto rnd = [&]() { x = x * 1664525u + 1013904223u; return ((x >> 8) * (1.f / 16777216.f) - 0.5f); };
  for (auto& v : hgi) v = rnd();
  for (auto& v : hw) v = 0.1f * rnd();
  for (auto& v : hb) v = 0.1f * rnd();
  float *gi, *w, *bh, *hL, *sv;
  hipMalloc(&gi, hgi.size() * 4);
  hipMalloc(&w, hw.size() * 4);
  hipMalloc(&bh, hb.size() * 4);
  hipMalloc(&hL, n1 * 4);
  hipMalloc(&sv, 4 * n1 * 4);
  hipMemcpy(gi, hgi.data(), hgi.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(bh, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  struct R { const char* name; float us; };
  R rs[] = {
      {"as shipped", time_fwd<0>(gi, w, bh, hL, sv, B, T, nd)},
      {"no MFMA", time_fwd<1>(gi, w, bh, hL, sv, B, T, nd)},
      {"no gate nonlinearities", time_fwd<2>(gi, w, bh, hL, sv, B, T, nd)},
      {"no global stores", time_fwd<4>(gi, w, bh, hL, sv, B, T, nd)},
      {"no barrier", time_fwd<8>(gi, w, bh, hL, sv, B, T, nd)},
      {"no gi loads", time_fwd<16>(gi, w, bh, hL, sv, B, T, nd)},
      {"no stores, no gi loads", time_fwd<20>(gi, w, bh, hL, sv, B, T, nd)},
      {"no MFMA, no nonlinearities", time_fwd<3>(gi, w, bh, hL, sv, B, T, nd)},
      {"MFMA only (no nonlin, stores, barrier, loads)", time_fwd<30>(gi, w, bh, hL, sv, B, T, nd)},
      {"nothing but the loop (all removed)", time_fwd<31>(gi, w, bh, hL, sv, B, T, nd)},
  };
  // the split-order step against the shipped one: same time, bitwise the same h / saved gates?
  std::vector<float> h1(n1), s1(4 * n1), h2(n1), s2(4 * n1);
  const float t0 = time_fwd<0>(gi, w, bh, hL, sv, B, T, nd);
  hipMemcpy(h1.data(), hL, n1 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(s1.data(), sv, 4 * n1 * 4, hipMemcpyDeviceToHost);
  const float t1 = time_fwd<0, true>(gi, w, bh, hL, sv, B, T, nd);
  hipMemcpy(h2.data(), hL, n1 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(s2.data(), sv, 4 * n1 * 4, hipMemcpyDeviceToHost);
  size_t diff = 0;
  for (size_t i = 0; i < n1; ++i) diff += memcmp(&h1[i], &h2[i], 4) != 0;
  for (size_t i = 0; i < 4 * n1; ++i) diff += memcmp(&s1[i], &s2[i], 4) != 0;
  printf("split order: %8.1f us (shipped %8.1f us), %zu differing floats of %zu\n", t1, t0, diff, 5 * n1);
  printf("split order, no stores: %8.1f us; no nonlinearities: %8.1f us\n",
         time_fwd<4, true>(gi, w, bh, hL, sv, B, T, nd), time_fwd<2, true>(gi, w, bh, hL, sv, B, T, nd));
  for (const R& r : rs) printf("%-48s %8.1f us  %6.2f us/step\n", r.name, r.us, r.us / T);
  return 0;
}
