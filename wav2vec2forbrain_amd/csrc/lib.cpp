// Library-level C ABI: error reporting, version, launch timing.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <mutex>
#include <vector>
#include "../../include/b2p_hip.h"
#include "timing.h"

static thread_local char g_err[1024] = "";

void b2p_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* b2p_last_error(void) { return g_err; }

// device counter mixed into every dropout seed (graph replays); NULL = eager semantics
static const uint64_t* g_seed_epoch = nullptr;
const uint64_t* b2p_seed_epoch() { return g_seed_epoch; }
extern "C" int b2p_set_seed_epoch(const uint64_t* dev_counter) {
  g_seed_epoch = dev_counter;
  return 0;
}
// LayerDrop gate of the layer being issued (device int, 0 = this replay skips the layer); NULL =
// ungated. Read by the GEMM and fused-attention launchers into their kernel arguments.
static const int32_t* g_gate = nullptr;
const int32_t* b2p_gate() { return g_gate; }
extern "C" int b2p_set_gate(const int32_t* dev_flag) {
  g_gate = dev_flag;
  return 0;
}
static const int64_t* g_gate_batch = nullptr;
const int64_t* b2p_gate_batch() { return g_gate_batch; }
extern "C" int b2p_set_gate_batch(const int64_t* dev_gate_ptrs) {
  g_gate_batch = dev_gate_ptrs;
  return 0;
}
extern "C" int b2p_version(void) { return 1; }
extern "C" int b2p_abi_sizes(int64_t* out3) {
  if (!out3) {
    b2p_set_error("abi_sizes: NULL");
    return 1;
  }
  out3[0] = (int64_t)sizeof(b2p_operand);
  out3[1] = (int64_t)sizeof(b2p_epilogue);
  out3[2] = (int64_t)sizeof(b2p_gemm_desc);
  return 0;
}

// ------------------------------------------------------------------ timing
namespace {
constexpr int kFamilies = 16;
struct Family {
  bool on = false;
  int max = 0;
  int used = 0;  // event pairs recorded
  std::vector<hipEvent_t> ev;  // 2 per launch
  std::vector<double> flops;
};
Family g_fam[kFamilies];
std::mutex g_mu;
}  // namespace

void b2p_timing_begin(int family, hipStream_t st) {
  if (family <= 0 || family >= kFamilies) return;
  Family& f = g_fam[family];
  if (!f.on || f.used >= f.max) return;
  hipEventRecord(f.ev[2 * f.used], st);
}

void b2p_timing_end(int family, hipStream_t st, double flops) {
  if (family <= 0 || family >= kFamilies) return;
  Family& f = g_fam[family];
  if (!f.on || f.used >= f.max) return;
  hipEventRecord(f.ev[2 * f.used + 1], st);
  f.flops[f.used] = flops;
  ++f.used;
}

extern "C" int b2p_timing_enable(int family, int max_events) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (family <= 0 || family >= kFamilies) {
    b2p_set_error("timing: family %d out of range", family);
    return 1;
  }
  Family& f = g_fam[family];
  for (auto e : f.ev) hipEventDestroy(e);
  f.ev.clear();
  f.flops.clear();
  f.used = 0;
  f.on = max_events > 0;
  f.max = max_events > 0 ? max_events : 0;
  if (!f.on) return 0;
  f.ev.resize(2 * (size_t)f.max);
  f.flops.resize(f.max);
  for (auto& e : f.ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      b2p_set_error("timing: hipEventCreate failed");
      return 2;
    }
  }
  return 0;
}

extern "C" int b2p_timing_read(int family, float* total_ms, int* count, double* total_flops) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (family <= 0 || family >= kFamilies) {
    b2p_set_error("timing: family %d out of range", family);
    return 1;
  }
  Family& f = g_fam[family];
  float tot = 0.f;
  double fl = 0.0;
  for (int i = 0; i < f.used; ++i) {
    if (hipEventSynchronize(f.ev[2 * i + 1]) != hipSuccess) {
      b2p_set_error("timing: event sync failed");
      return 2;
    }
    float ms = 0.f;
    hipEventElapsedTime(&ms, f.ev[2 * i], f.ev[2 * i + 1]);
    tot += ms;
    fl += f.flops[i];
  }
  if (total_ms) *total_ms = tot;
  if (count) *count = f.used;
  if (total_flops) *total_flops = fl;
  return 0;
}
