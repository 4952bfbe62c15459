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

// the update of one tensor's elements (grid-strided over blockIdx.x); every form of the kernel runs
// this same code, so host-form, device-form and gated updates are bit-identical for equal inputs
__device__ __forceinline__ void adam_range(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                           float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                                           float wd, float bc1, float bc2s) {
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

__global__ void __launch_bounds__(NTH) adam_k(const int64_t* __restrict__ table, float lr, float b1, float b2,
                                              float eps, float wd, float bc1, float bc2s,
                                              const float* __restrict__ hyper) {
  if (hyper) {   // graph-replayable form: lr and the bias corrections live on the device
    lr = hyper[0];
    bc1 = hyper[1];
    bc2s = hyper[2];
  }
  const int64_t* rec = table + 5 * (int64_t)blockIdx.y;
  adam_range(reinterpret_cast<float*>(rec[0]), reinterpret_cast<const float*>(rec[1]), reinterpret_cast<float*>(rec[2]),
             reinterpret_cast<float*>(rec[3]), rec[4], lr, b1, b2, eps, wd, bc1, bc2s);
}
// one thread: the step counter of a parameter group and its bias corrections (double, as the host
// computes them for torch.optim.Adam), for a step captured in a graph
__global__ void adam_hyper_k(double* __restrict__ st, const float* __restrict__ lr, double b1, double b2,
                             float* __restrict__ hyper) {
  const double t = st[0] + 1.0;
  st[0] = t;
  hyper[0] = lr[0];
  hyper[1] = (float)(1.0 - pow(b1, t));
  hyper[2] = (float)sqrt(1.0 - pow(b2, t));
}

__global__ void epoch_step_k(uint64_t* c) { c[0] += 1; }

// the same update with the tensor records passed by value in the kernel arguments (no device table:
// nothing to upload, and a captured graph keeps the records in its kernel node)
constexpr int ADAM_MAXR = 48;
struct AdamRecs {
  int64_t r[ADAM_MAXR][5];   // param, grad, exp_avg, exp_avg_sq, numel
};
__global__ void __launch_bounds__(NTH) adam_rec_k(const AdamRecs recs, float lr, float b1, float b2, float eps,
                                                  float wd, float bc1, float bc2s, const float* __restrict__ hyper) {
  if (hyper) {
    lr = hyper[0];
    bc1 = hyper[1];
    bc2s = hyper[2];
  }
  const int64_t* rec = recs.r[blockIdx.y];
  adam_range(reinterpret_cast<float*>(rec[0]), reinterpret_cast<const float*>(rec[1]), reinterpret_cast<float*>(rec[2]),
             reinterpret_cast<float*>(rec[3]), rec[4], lr, b1, b2, eps, wd, bc1, bc2s);
}

// Per-tensor step counters and gates (the device form HipAdam uses for captured and DP steps).
// torch.optim.Adam leaves a parameter whose .grad is None untouched: no moment update, no weight
// decay, no step increment (src/experiments/experiment.py:25-28). Under LayerDrop the reference's
// skipped layers are exactly such parameters; a captured step runs every layer and marks a skipped
// one with its gate flag, so a closed gate here reproduces the None-grad skip.
constexpr int GADAM_MAXR = 32;
struct GatedAdamRecs {
  int64_t r[GADAM_MAXR][7];   // param, grad, exp_avg, exp_avg_sq, numel, step (double*), gate (int32*)
};
// one thread per record: advance the step of an open tensor and form its bias corrections in double,
// rounded to float as the host form passes them (bit-identical updates in both forms); hyper[i] =
// {lr, bc1, sqrt(bc2), open}, open = 0 for a closed gate
__global__ void adam_gate_steps_k(const GatedAdamRecs recs, int nrec, const float* __restrict__ lr_dev, double b1,
                                  double b2, float4* __restrict__ hyper) {
  const int i = threadIdx.x;
  if (i >= nrec) return;
  const int64_t* rec = recs.r[i];
  const int32_t* gate = reinterpret_cast<const int32_t*>(rec[6]);
  if (gate != nullptr && *gate == 0) {
    hyper[i] = make_float4(0.f, 1.f, 1.f, 0.f);
    return;
  }
  double* st = reinterpret_cast<double*>(rec[5]);
  const double t = st[0] + 1.0;
  st[0] = t;
  hyper[i] = make_float4(lr_dev[0], (float)(1.0 - pow(b1, t)), (float)sqrt(1.0 - pow(b2, t)), 1.f);
}
__global__ void __launch_bounds__(NTH) adam_gated_k(const GatedAdamRecs recs, float b1, float b2, float eps,
                                                    float wd, const float4* __restrict__ hyper) {
  const float4 h = hyper[blockIdx.y];
  if (h.w == 0.f) return;   // gate closed: parameter, moments and step stay as they are
  const int64_t* rec = recs.r[blockIdx.y];
  adam_range(reinterpret_cast<float*>(rec[0]), reinterpret_cast<const float*>(rec[1]), reinterpret_cast<float*>(rec[2]),
             reinterpret_cast<float*>(rec[3]), rec[4], h.x, b1, b2, eps, wd, h.y, h.z);
}

// gradient accumulation over many small tensors in one launch (records by value: capturable, nothing
// uploaded). blockIdx.y = record, blockIdx.x strides its elements. Record {dst, src, numel, nrows,
// set}: dst[i] (set ? = : +=) sum_{r < nrows} src[r * numel + i], rows summed in order — nrows 1 is
// the plain accumulation; nrows > 1 takes column sums still held as per-tile partial rows (a GEMM
// epilogue's or b2p_drop_cast_colsum's) and finishes them here, on the side stream.
constexpr int ACC_MAXR = 64;
struct AccRecs {
  int64_t r[ACC_MAXR][5];   // dst, src, numel, nrows, set
};
__global__ void __launch_bounds__(NTH) accum_rec_k(const AccRecs recs) {
  const int64_t* rec = recs.r[blockIdx.y];
  float* __restrict__ dst = reinterpret_cast<float*>(rec[0]);
  const float* __restrict__ src = reinterpret_cast<const float*>(rec[1]);
  const int64_t n = rec[2], nrows = rec[3];
  const bool set = rec[4] != 0;
  const int64_t stride = (int64_t)gridDim.x * NTH;
  for (int64_t i = (int64_t)blockIdx.x * NTH + threadIdx.x; i < n; i += stride) {
    // rows in order, 8 loads in flight per step (the partial rows are ~60-130 deep)
    float v = src[i];
    int64_t r = 1;
    for (; r + 8 <= nrows; r += 8) {
      float q[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = src[(r + k) * n + i];
#pragma unroll
      for (int k = 0; k < 8; ++k) v += q[k];
    }
    for (; r < nrows; ++r) v += src[r * n + i];
    dst[i] = set ? v : dst[i] + v;
  }
}

int accum_launch(const int64_t* recs, int width, int ntensors, hipStream_t st) {
  for (int c0 = 0; c0 < ntensors; c0 += ACC_MAXR) {
    const int nc = ntensors - c0 < ACC_MAXR ? ntensors - c0 : ACC_MAXR;
    AccRecs a;
    int64_t maxn = 0, maxr = 1;
    for (int i = 0; i < nc; ++i) {
      const int64_t* q = recs + (int64_t)width * (c0 + i);
      a.r[i][0] = q[0];
      a.r[i][1] = q[1];
      a.r[i][2] = q[2];
      a.r[i][3] = width == 5 ? q[3] : 1;
      a.r[i][4] = width == 5 ? q[4] : 0;
      B2P_CHECK_ARG(a.r[i][2] <= 0 || (a.r[i][0] && a.r[i][1]), "accum_recs: NULL tensor in a record");
      B2P_CHECK_ARG(a.r[i][3] >= 1, "accum_recs: nrows must be >= 1");
      maxn = a.r[i][2] > maxn ? a.r[i][2] : maxn;
      maxr = a.r[i][3] > maxr ? a.r[i][3] : maxr;
    }
    if (maxn <= 0) continue;
    // row-summing records: one element per thread (their cost is the row loop, not the width)
    const int64_t per = maxr > 1 ? 1 : PER_THREAD;
    int64_t bx = (maxn + (int64_t)NTH * per - 1) / ((int64_t)NTH * per);
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(accum_rec_k, dim3((unsigned)bx, (unsigned)nc), dim3(NTH), 0, st, a);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}
}  // namespace

extern "C" int b2p_seed_epoch_step(uint64_t* dev_counter, b2p_stream_t stream) {
  B2P_CHECK_ARG(dev_counter != nullptr, "seed_epoch_step: NULL counter");
  hipLaunchKernelGGL(epoch_step_k, dim3(1), dim3(1), 0, (hipStream_t)stream, dev_counter);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_adam_recs(const int64_t* recs, int ntensors, float lr, double beta1, double beta2, float eps,
                             float weight_decay, float bias_c1, float bias_c2_sqrt, const float* lr_dev,
                             double* step_dev, float* hyper_dev, b2p_stream_t stream) {
  B2P_CHECK_ARG(recs != nullptr || ntensors == 0, "adam_recs: NULL records");
  B2P_CHECK_ARG(ntensors >= 0, "adam_recs: bad tensor count");
  const bool dev = step_dev != nullptr;
  B2P_CHECK_ARG(!dev || (lr_dev && hyper_dev), "adam_recs: device form needs lr_dev, step_dev and hyper_dev");
  B2P_CHECK_ARG(dev || (bias_c1 > 0.f && bias_c2_sqrt > 0.f), "adam: bias corrections must be positive");
  hipStream_t st = (hipStream_t)stream;
  if (dev) hipLaunchKernelGGL(adam_hyper_k, dim3(1), dim3(1), 0, st, step_dev, lr_dev, beta1, beta2, hyper_dev);
  const float b1f = (float)beta1, b2f = (float)beta2;
  for (int c0 = 0; c0 < ntensors; c0 += ADAM_MAXR) {
    const int nc = ntensors - c0 < ADAM_MAXR ? ntensors - c0 : ADAM_MAXR;
    AdamRecs a;
    int64_t maxn = 0;
    for (int i = 0; i < nc; ++i) {
      for (int k = 0; k < 5; ++k) a.r[i][k] = recs[5 * (c0 + i) + k];
      maxn = a.r[i][4] > maxn ? a.r[i][4] : maxn;
    }
    if (maxn <= 0) continue;
    int64_t bx = (maxn + (int64_t)NTH * PER_THREAD - 1) / ((int64_t)NTH * PER_THREAD);
    if (bx > 4096) bx = 4096;
    hipLaunchKernelGGL(adam_rec_k, dim3((unsigned)bx, (unsigned)nc), dim3(NTH), 0, st, a, lr, b1f, b2f, eps,
                       weight_decay, bias_c1, bias_c2_sqrt, dev ? (const float*)hyper_dev : nullptr);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_adam_gated_recs(const int64_t* recs, int ntensors, const float* lr_dev, double beta1,
                                   double beta2, float eps, float weight_decay, float* hyper_dev,
                                   b2p_stream_t stream) {
  B2P_CHECK_ARG(recs != nullptr || ntensors == 0, "adam_gated_recs: NULL records");
  B2P_CHECK_ARG(ntensors >= 0, "adam_gated_recs: bad tensor count");
  B2P_CHECK_ARG(ntensors == 0 || (lr_dev && hyper_dev), "adam_gated_recs: NULL lr_dev / hyper_dev");
  hipStream_t st = (hipStream_t)stream;
  const float b1f = (float)beta1, b2f = (float)beta2;
  for (int c0 = 0; c0 < ntensors; c0 += GADAM_MAXR) {
    const int nc = ntensors - c0 < GADAM_MAXR ? ntensors - c0 : GADAM_MAXR;
    GatedAdamRecs a;
    int64_t maxn = 0;
    for (int i = 0; i < nc; ++i) {
      for (int k = 0; k < 7; ++k) a.r[i][k] = recs[7 * (c0 + i) + k];
      B2P_CHECK_ARG(a.r[i][5] != 0, "adam_gated_recs: NULL step counter in a record");
      B2P_CHECK_ARG(a.r[i][4] <= 0 || (a.r[i][0] && a.r[i][1] && a.r[i][2] && a.r[i][3]),
                    "adam_gated_recs: NULL tensor in a record");
      maxn = a.r[i][4] > maxn ? a.r[i][4] : maxn;
    }
    float4* hy = reinterpret_cast<float4*>(hyper_dev) + c0;
    hipLaunchKernelGGL(adam_gate_steps_k, dim3(1), dim3(64), 0, st, a, nc, lr_dev, beta1, beta2, hy);
    if (maxn <= 0) continue;
    int64_t bx = (maxn + (int64_t)NTH * PER_THREAD - 1) / ((int64_t)NTH * PER_THREAD);
    if (bx > 4096) bx = 4096;
    hipLaunchKernelGGL(adam_gated_k, dim3((unsigned)bx, (unsigned)nc), dim3(NTH), 0, st, a, b1f, b2f, eps,
                       weight_decay, (const float4*)hy);
  }
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_adam_multi_dev(const int64_t* table, int ntensors, int64_t max_numel, const float* lr_dev,
                                  float beta1, float beta2, float eps, float weight_decay, double* step_dev,
                                  float* hyper_dev, b2p_stream_t stream) {
  B2P_CHECK_ARG(table && lr_dev && step_dev && hyper_dev, "adam_dev: NULL pointer");
  B2P_CHECK_ARG(ntensors >= 0 && ntensors < 65536, "adam: bad tensor count");
  hipLaunchKernelGGL(adam_hyper_k, dim3(1), dim3(1), 0, (hipStream_t)stream, step_dev, lr_dev, (double)beta1,
                     (double)beta2, hyper_dev);
  if (ntensors == 0 || max_numel <= 0) return 0;
  int64_t bx = (max_numel + (int64_t)NTH * PER_THREAD - 1) / ((int64_t)NTH * PER_THREAD);
  if (bx > 4096) bx = 4096;
  hipLaunchKernelGGL(adam_k, dim3((unsigned)bx, (unsigned)ntensors), dim3(NTH), 0, (hipStream_t)stream, table, 0.f,
                     beta1, beta2, eps, weight_decay, 1.f, 1.f, (const float*)hyper_dev);
  B2P_CHECK_LAUNCH();
  return 0;
}

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
                     beta1, beta2, eps, weight_decay, bias_c1, bias_c2_sqrt, (const float*)nullptr);
  B2P_CHECK_LAUNCH();
  return 0;
}

extern "C" int b2p_accum_recs(const int64_t* recs, int ntensors, b2p_stream_t stream) {
  B2P_CHECK_ARG(recs != nullptr || ntensors == 0, "accum_recs: NULL records");
  B2P_CHECK_ARG(ntensors >= 0, "accum_recs: bad tensor count");
  return accum_launch(recs, 3, ntensors, (hipStream_t)stream);
}

extern "C" int b2p_accum_rows_recs(const int64_t* recs, int ntensors, b2p_stream_t stream) {
  B2P_CHECK_ARG(recs != nullptr || ntensors == 0, "accum_rows_recs: NULL records");
  B2P_CHECK_ARG(ntensors >= 0, "accum_rows_recs: bad tensor count");
  return accum_launch(recs, 5, ntensors, (hipStream_t)stream);
}
