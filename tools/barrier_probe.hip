// Cost of a workgroup barrier on gfx950: one block per CU (LDS-limited), NB barriers
// per iteration, timed with HIP events; prints ns per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int NB>
__global__ __launch_bounds__(1024) void bar_kernel(int iters, float* out) {
  __shared__ float pad[35000];   // ~140 KB: one block per CU
  float acc = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    acc += 1.0f;
  }
  pad[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = pad[(threadIdx.x + 1) & 1023];
}
template <int NB>
float run(int threads, int iters, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  bar_kernel<NB><<<256, threads>>>(iters, out);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) bar_kernel<NB><<<256, threads>>>(iters, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}
int main() {
  float* out; hipMalloc(&out, 4096);
  const int its[2] = {1280, 128000};
  for (int threads : {512, 1024})
    for (int it : its) {
      float t0 = run<0>(threads, it, out), t1 = run<1>(threads, it, out), t2 = run<2>(threads, it, out);
      printf("threads %4d iters %6d: 0 bar %.4f ms, 1 bar %.4f ms, 2 bar %.4f ms -> %.1f ns per barrier\n",
             threads, it, t0, t1, t2, (t2 - t1) * 1e6 / it);
    }
  return 0;
}
