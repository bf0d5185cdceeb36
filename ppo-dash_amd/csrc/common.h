// Shared helpers for libppo_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "../../include/ppo_hip.h"  // every PPO_API definition must match its declaration

#define PPO_API extern "C" __attribute__((visibility("default")))

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Exact three-way bf16 split of an fp32 value: v == hi + mid + lo (each part
// rounded to nearest-even from the remaining residual; 3 x 8 significand bits
// cover fp32's 24).  Used where one GEMM operand is exactly representable in
// bf16 (u8 pixels): every bf16 x bf16 product is then exact in fp32 and the
// MFMA accumulates in fp32, i.e. fp32 arithmetic on the bf16 matrix cores.
__host__ __device__ __forceinline__ uint32_t bf16_rne_bits(float v) {
  uint32_t u;
  memcpy(&u, &v, 4);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__host__ __device__ __forceinline__ float bf16_bits_to_f32(uint32_t h) {
  const uint32_t u = h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
__host__ __device__ __forceinline__ void split_bf16x3(float v, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  hi = bf16_rne_bits(v);
  const float r1 = v - bf16_bits_to_f32(hi);
  mid = bf16_rne_bits(r1);
  const float r2 = r1 - bf16_bits_to_f32(mid);
  lo = bf16_rne_bits(r2);
}

// Error plumbing: every C-ABI entry point returns 0 on success, a hipError_t
// value or a library code otherwise; ppo_last_error() returns the message.
void ppo_set_error(const char* fmt, ...);

#define PPO_REQUIRE(cond, ...)                                                       \
  do {                                                                               \
    if (!(cond)) {                                                                   \
      ppo_set_error(__VA_ARGS__);                                                    \
      return PPO_EARG;                                                               \
    }                                                                                \
  } while (0)

#define PPO_LAUNCH_CHECK(name)                                                       \
  do {                                                                               \
    hipError_t _e = hipGetLastError();                                               \
    if (_e != hipSuccess) {                                                          \
      ppo_set_error("%s: launch failed: %s", name, hipGetErrorString(_e));           \
      return (int)_e;                                                                \
    }                                                                                \
  } while (0)

#define PPO_HIP_CHECK(expr, name)                                                    \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      ppo_set_error("%s: %s", name, hipGetErrorString(_e));                          \
      return (int)_e;                                                                \
    }                                                                                \
  } while (0)

// Launch-level event profiler (bench.py roofline): launches whose name matches
// the enabled one are bracketed by hipEventRecord on their stream and tagged
// with their algorithmic FLOP (or byte) count.
bool ppo_prof_begin(const char* name, hipStream_t st, int* slot);
void ppo_prof_end(int slot, hipStream_t st, double work);

// the same for a whole API call (all launches it makes): events at entry and exit
struct ProfScope {
  hipStream_t st;
  double work;
  int slot = -1;
  bool on;
  ProfScope(const char* name, hipStream_t s, double w) : st(s), work(w) { on = ppo_prof_begin(name, s, &slot); }
  ~ProfScope() {
    if (on) ppo_prof_end(slot, st, work);
  }
};

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline unsigned ceil_div(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// workgroup barrier publishing LDS writes (lgkmcnt(0)) as one asm statement, for
// the kernels that stage LDS by DMA (global_load_lds, asm) and wait for it with
// their own vmcnt counts.  On gfx950 __syncthreads emits the same two instructions
// (its workgroup fence adds no vmcnt wait: loads in flight stay in flight), so
// elsewhere the two are interchangeable.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One 1-KB LDS-DMA piece: lane i's 16 B from gsrc land at LDS byte lds_dst + 16 i
// (inline asm: invisible to the compiler's waitcnt pass, so every user retires it
// with its own vmcnt count, stated at the use)
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// Range-checked buffer stores: a store whose byte offset is out of the
// resource's range (e.g. -1) is dropped by the hardware — predication without an
// exec-mask branch.  dword3 0x00020000: raw 32-bit buffer on gfx9 (gfx950).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void bstore_f32(float v, __amdgpu_buffer_rsrc_t r, int off_bytes) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off_bytes, 0, 0);
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bstore_f32x4(f32x4 v, __amdgpu_buffer_rsrc_t r, int off_bytes) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, off_bytes, 0, 0);
}

// u8 -> fp32 decode, bit-identical to (float)u / 255.0f (IEEE divide), which is
// the oracle's input convention u8.float()/255.0.  q = u*(1/255)
// is wrong for 126 of the 256 codes; one residual FMA correction makes all 256
// exact (checked exhaustively on the host, tests/test_host_logic.py).
__device__ __forceinline__ float decode_u8(uint32_t u) {
  const float r = 1.0f / 255.0f;
  const float x = (float)u;
  const float q = x * r;
  const float res = __builtin_fmaf(-q, 255.0f, x);
  return __builtin_fmaf(res, r, q);
}

// Counter-based hash RNG (splitmix64 finaliser) for the device sampling noise
// and the synthetic environment.
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// uniform in (0, 1]: 24 random bits
__host__ __device__ __forceinline__ float u01_open0(uint64_t h) {
  return ((float)((uint32_t)(h >> 40)) + 1.0f) * (1.0f / 16777216.0f);
}
