// Optional HIP-event timing of tagged kernel launches (bench.py roofline). Off by default:
// when a family is not enabled, begin/end are a single branch.
#pragma once
#include <hip/hip_runtime.h>

void b2p_timing_begin(int family, hipStream_t st);
void b2p_timing_end(int family, hipStream_t st, double flops);
