// Microbenchmark of the GEMM core's inner-loop ingredients on gfx950 fp32 MFMA
// (v_mfma_f32_32x32x2_f32): which part of a k-step costs MFMA issue slots.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
// Each variant runs a 128x128-tile-like wave workload: 4 waves / block, each
// wave 4 accumulators (2x2 tiles of 32x32), 32 MFMAs per "k-step".
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

// MODE 0: MFMA only (register operands)
// MODE 1: + 8 ds_read_b128 per k-step (4 per 16 MFMAs), no barrier
// MODE 2: + one __syncthreads per k-step
// MODE 3: + 4 ds_write_b128 per k-step (staging into the other buffer)
// MODE 4: + 4 global_load_dwordx4 per k-step (L2-resident source)
// MODE 5: 4 global_load_lds_dwordx4 per k-step instead of loads + ds_write, barrier per step
// MODE 6: MODE 4 with two k-steps (64 MFMAs) per barrier
// MODE 7: MODE 5 with two k-steps (64 MFMAs) per barrier
template <int MODE>
__global__ __launch_bounds__(256) void probe(const float* __restrict__ src, float* __restrict__ out, int steps) {
  __shared__ __attribute__((aligned(16))) float smem[2 * 2 * 128 * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 2 * 2 * 128 * 16; i += 256) smem[i] = (float)(i & 7) * 0.001f;
  __syncthreads();
  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f32x4 af[2], bf[2];
  for (int i = 0; i < 2; ++i) { af[i] = f32x4{1.f, 2.f, 3.f, 4.f} * (float)(lane + 1); bf[i] = af[i] * 0.5f; }
  f32x4 ld[4];
  const f32x4* g = reinterpret_cast<const f32x4*>(src) + (blockIdx.x & 255) * 1024 + tid;
  constexpr bool GLDS = MODE == 5 || MODE == 7;
  constexpr int PER_BAR = (MODE == 6 || MODE == 7) ? 2 : 1;
  for (int t = 0; t < steps; ++t) {
    const int buf = (t / PER_BAR) & 1;
    if (MODE >= 4 && !GLDS) {
      for (int q = 0; q < 4; ++q) ld[q] = g[q * 256];
    }
    if (GLDS) {
      float* Ws = smem + (buf ^ 1) * 4096 + (t % PER_BAR) * 0;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g + q * 256),
                                         (__attribute__((address_space(3))) void*)(Ws + (q * 256 + wave * 64) * 4),
                                         16, 0, 0);
    }
    const float* As = smem + buf * 4096;
#pragma unroll
    for (int kk = 0; kk < 16; kk += 8) {
      if (MODE >= 1) {
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const f32x4*>(As + ((wave & 1) * 64 + i * 32 + (lane & 31)) * 16 + kk + 4 * (lane >> 5));
        for (int j = 0; j < 2; ++j)
          bf[j] = *reinterpret_cast<const f32x4*>(As + 2048 + ((wave >> 1) * 64 + j * 32 + (lane & 31)) * 16 + kk + 4 * (lane >> 5));
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    if (MODE >= 3 && !GLDS) {
      float* Ws = smem + (buf ^ 1) * 4096;
      for (int q = 0; q < 4; ++q) {
        f32x4 v = MODE >= 4 ? ld[q] : af[q & 1];
        *reinterpret_cast<f32x4*>(Ws + (q * 256 + tid) * 4) = v;
      }
    }
    if (MODE >= 2 && (t % PER_BAR) == PER_BAR - 1) __syncthreads();
  }
  float s = 0.f;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  out[blockIdx.x * 256 + tid] = s;
}

template <int MODE>
int run(const float* src, float* out, int blocks, int steps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  probe<MODE><<<blocks, 256>>>(src, out, steps);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  probe<MODE><<<blocks, 256>>>(src, out, steps);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double flops = 2.0 * 32 * 32 * 2 * 32.0 * steps * 4 * blocks;   // 32 MFMAs x 4 waves per step
  printf("mode %d blocks %5d: %8.3f ms  %6.1f TFLOP/s\n", MODE, blocks, ms, flops / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  float *src, *out;
  CHECK(hipMalloc(&src, 256 * 1024 * 16 * 4));
  CHECK(hipMemset(src, 0, 256 * 1024 * 16 * 4));
  CHECK(hipMalloc(&out, 4096 * 256 * 4));
  const int steps = 2000;
  for (int blocks : {512, 768, 1024}) {
    if (run<0>(src, out, blocks, steps)) return 1;
    if (run<1>(src, out, blocks, steps)) return 1;
    if (run<2>(src, out, blocks, steps)) return 1;
    if (run<3>(src, out, blocks, steps)) return 1;
    if (run<4>(src, out, blocks, steps)) return 1;
    if (run<5>(src, out, blocks, steps)) return 1;
    if (run<6>(src, out, blocks, steps)) return 1;
    if (run<7>(src, out, blocks, steps)) return 1;
  }
  return 0;
}
