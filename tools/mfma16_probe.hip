// Does a VALU-produced MFMA operand (u8 -> f32 convert right before each
// v_mfma_f32_16x16x4_f32) cost matrix-core throughput on gfx950?
//   hipcc -O3 --offload-arch=gfx950 tools/mfma16_probe.hip -o tools/mfma16_probe.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ f32x4 cvt4(uint32_t u) {
  return f32x4{(float)(u & 255u), (float)((u >> 8) & 255u), (float)((u >> 16) & 255u), (float)(u >> 24)};
}

// MODE 0: register operands.  MODE 1: A fragment = cvt of a loop-varying u32.
// MODE 2: MODE 1 + the u32 from a ds_read_b32 per fragment.
// MODE 3: MODE 2 with all 13 fragments converted before the MFMA burst.
template <int MODE>
__global__ __launch_bounds__(512) void probe(float* out, int steps) {
  __shared__ uint32_t lds[8192];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 8192; i += 512) lds[i] = i * 2654435761u;
  __syncthreads();
  f32x4 acc[13];
  for (int t = 0; t < 13; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 b = f32x4{1.f, 2.f, 3.f, 4.f} * (float)lane;
  uint32_t u = lane * 0x01020304u;
  for (int it = 0; it < steps; ++it) {
    if (MODE == 3) {
      f32x4 a[13];
#pragma unroll
      for (int t = 0; t < 13; ++t) a[t] = cvt4(lds[(it * 13 + t * 64 + lane) & 8191]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int t = 0; t < 13; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][s], b[s], acc[t], 0, 0, 0);
    } else {
#pragma unroll
      for (int t = 0; t < 13; ++t) {
        f32x4 a;
        if (MODE == 0) a = b * 0.5f;
        else if (MODE == 1) a = cvt4(u + t + it);
        else a = cvt4(lds[(it * 13 + t * 64 + lane) & 8191]);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc[t], 0, 0, 0);
      }
    }
  }
  float sum = 0.f;
  for (int t = 0; t < 13; ++t) sum += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
  out[blockIdx.x * 512 + tid] = sum;
}

template <int MODE>
int run(float* out, int blocks, int steps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  probe<MODE><<<blocks, 512>>>(out, steps);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  probe<MODE><<<blocks, 512>>>(out, steps);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double flops = 2.0 * 16 * 16 * 4 * 52.0 * steps * 8 * blocks;
  printf("mode %d blocks %4d: %8.3f ms  %6.1f TFLOP/s\n", MODE, blocks, ms, flops / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  float* out;
  CHECK(hipMalloc(&out, 1024 * 512 * 4));
  for (int blocks : {256, 512}) {
    if (run<0>(out, blocks, 4000) || run<1>(out, blocks, 4000) || run<2>(out, blocks, 4000) ||
        run<3>(out, blocks, 4000))
      return 1;
  }
  return 0;
}
