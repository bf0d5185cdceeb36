// MFMA issue-rate probe (gfx950): back-to-back v_mfma_f32_16x16x32_bf16 vs
// v_mfma_f32_16x16x16_bf16 vs v_mfma_f32_32x32x16_bf16 on 4 independent accumulators,
// one wave per SIMD, random-ish operands; prints cycles per instruction (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o /tmp/mfma_rate && /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int N = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc, float seed) {
  const int l = threadIdx.x;
  bf16x8 a8, b8;
  bf16x4 a4, b4;
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(seed * (l + i)); b8[i] = (__bf16)(seed * (l - i)); }
  for (int i = 0; i < 4; ++i) { a4[i] = a8[i]; b4[i] = b8[i]; }
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  f32x16 d0 = {}, d1 = {};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < N; ++it) {
    if constexpr (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, c3, 0, 0, 0);
    } else if constexpr (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, c3, 0, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d1, 0, 0, 0);
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, d1, 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  for (int i = 0; i < 16; ++i) s += d0[i] + d1[i];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, int flop_per) {
  float* out; long long* cyc;
  const int nb = 256;
  hipMalloc(&out, nb * 256 * 4); hipMalloc(&cyc, nb * 8);
  probe<KIND><<<nb, 256>>>(out, cyc, 0.001f);   // warm
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) probe<KIND><<<nb, 256>>>(out, cyc, 0.001f);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long h[nb]; hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double avg = 0; for (int i = 0; i < nb; ++i) avg += h[i]; avg /= nb;
  const double insts = 4.0 * N;   // per wave
  const double tflops = 5.0 * nb * 4 * insts * flop_per / (ms * 1e-3) / 1e12;
  printf("%-28s %7.2f cyc/inst (s_memtime, per wave, 1 wave/SIMD)  %8.1f TFLOP/s  %.3f ms\n", name, avg / insts, tflops, ms / 5);
  hipFree(out); hipFree(cyc);
}

int main() {
  run<0>("mfma_f32_16x16x32_bf16", 2 * 16 * 16 * 32);
  run<1>("mfma_f32_16x16x16_bf16", 2 * 16 * 16 * 16);
  run<2>("mfma_f32_32x32x16_bf16", 2 * 32 * 32 * 16);
  run<0>("mfma_f32_16x16x32_bf16", 2 * 16 * 16 * 32);
  run<1>("mfma_f32_16x16x16_bf16", 2 * 16 * 16 * 16);
  return 0;
}
