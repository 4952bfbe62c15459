// Multi-tensor Adam with L2 weight decay (torch.optim.Adam semantics, as constructed in
// src/experiments/experiment.py:25-28 and src/experiments/b2t_gru_w2v_experiment.py:138-145):
//   g += wd * p ; m = lerp(m, g, 1-b1) ; v = b2 v + (1-b2) g^2
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// One launch updates every tensor of a parameter group: grid.y indexes a device table of
// {param, grad, exp_avg, exp_avg_sq, numel} records. HBM-bound: 28 B / element.
#include "common.h"
#include "../../include/b2p_hip.h"

namespace {
constexpr int NTH = 256;
constexpr int PER_THREAD = 4;

__global__ void __launch_bounds__(NTH) adam_k(const int64_t* __restrict__ table, float lr, float b1, float b2,
                                              float eps, float wd, float bc1, float bc2s) {
  const int64_t* rec = table + 5 * (int64_t)blockIdx.y;
  float* __restrict__ p = reinterpret_cast<float*>(rec[0]);
  const float* __restrict__ g = reinterpret_cast<const float*>(rec[1]);
  float* __restrict__ m = reinterpret_cast<float*>(rec[2]);
  float* __restrict__ v = reinterpret_cast<float*>(rec[3]);
  const int64_t n = rec[4];
  const float step = lr / bc1;
  const int64_t stride = (int64_t)gridDim.x * NTH;
  for (int64_t i = (int64_t)blockIdx.x * NTH + threadIdx.x; i < n; i += stride) {
    float gi = g[i];
    const float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    float vi = v[i];
    vi = b2 * vi + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2s + eps;
    p[i] = pi - step * (mi / denom);
  }
}
}  // namespace

extern "C" int b2p_adam_multi(const int64_t* table, int ntensors, int64_t max_numel, float lr, float beta1,
                              float beta2, float eps, float weight_decay, float bias_c1, float bias_c2_sqrt,
                              b2p_stream_t stream) {
  B2P_CHECK_ARG(table != nullptr, "adam: NULL table");
  B2P_CHECK_ARG(ntensors >= 0 && ntensors < 65536, "adam: bad tensor count");
  if (ntensors == 0 || max_numel <= 0) return 0;
  B2P_CHECK_ARG(bias_c1 > 0.f && bias_c2_sqrt > 0.f, "adam: bias corrections must be positive");
  int64_t bx = (max_numel + (int64_t)NTH * PER_THREAD - 1) / ((int64_t)NTH * PER_THREAD);
  if (bx > 4096) bx = 4096;
  hipLaunchKernelGGL(adam_k, dim3((unsigned)bx, (unsigned)ntensors), dim3(NTH), 0, (hipStream_t)stream, table, lr,
                     beta1, beta2, eps, weight_decay, bias_c1, bias_c2_sqrt);
  B2P_CHECK_LAUNCH();
  return 0;
}
