// Small-batch forward launchers (small.hip), internal to libppo_hip.so: the
// forward entry points of gemm.hip route B <= ppo_tune_get("small_b") here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

int small_conv1_fwd(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                    const float* w1, const float* b1, float* out, hipStream_t s);
int small_conv2_fwd(const float* a1, int B, const float* w2p, const float* b2, float* out, hipStream_t s);
int small_conv3_fwd(const float* a2, int B, const float* w3p, const float* b3, float* out, hipStream_t s);
int small_linear_fwd(const float* x, const int64_t* idx, int M, int K, int lda, const float* w, const float* b,
                     int N, float* out, int ldo, int act, hipStream_t s);
