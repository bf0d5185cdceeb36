// Observation boundary on the GPU: the env-side
// wrappers that turn a raw u8 RGB frame into the policy input, fused into one
// pass over the frame, and the device-side frame stack.
//
// Reference (ppo-dash-study/013_…/, the "norm_obs" variants; T/ has the same
// classes with the `if self.mean:` bug that raises on an ndarray):
//   NormalizeWrapper.observation   sohojoe_wrappers.py:872-884
//       x = (u8 - mean[y][x][c]) / std   (float64; mean/std from ObtRetro-v6_*.txt)
//       or x = u8 / 255                  (float64, no normaliser file)
//   FrameStackMono(k=2)._add_ob/_get_ob  sohojoe_wrappers.py:425-501
//       channels = R, G, B of the current frame + mono_frames[1], the current
//       frame's cv2 RGB2GRAY of x.astype(float32); np.array(frames).T transposes
//       the (H, W) mono image against the (W, H) colour planes, so the mono
//       channel at (y, x) is gray(frame[x][y]) — reproduced here (H == W).
//   TransposeImage op=[2,0,1]      pytorch_wrappers.py:170-203   HWC -> CHW
//   VecPyTorch.step_wait .float()  pytorch_wrappers.py:105-160   float64 -> fp32
//   VecPyTorchFrameStack           pytorch_wrappers.py:58-102
//       stacked[:, :-C] = stacked[:, C:]; stacked[i] = 0 where done; stacked[:, -C:] = obs
//
// Both kernels are HBM-bound streams (u8 in, fp32 out); one thread per pixel.
#include "common.h"

namespace {

constexpr int OBS_THREADS = 256;

// cv2 cvtColor(COLOR_RGB2GRAY) on float32: R*0.299f + G*0.587f + B*0.114f, summed
// left to right (OpenCV's RGB2Gray<float> scalar loop); this file is built with
// -ffp-contract=off (Makefile): hipcc's default contraction would fuse the last add
__device__ __forceinline__ float gray_f32(float r, float g, float b) {
  return __fadd_rn(__fadd_rn(__fmul_rn(r, 0.299f), __fmul_rn(g, 0.587f)), __fmul_rn(b, 0.114f));
}

// fl32(fl64(d / s)) without a float64 divide per element: q = d·(1/s) differs from
// the IEEE quotient by at most a few units of its last bit, so it rounds to the same
// fp32 unless the 29 bits the fp32 rounding drops lie within 4 units of the
// midpoint pattern — there the IEEE division decides (the same test conv1f.hip's
// fused decode uses; bit-identity with the reference chain: tests/test_obs_boundary.py)
__device__ __attribute__((noinline)) double obs_ieee_div(double d, double s) { return d / s; }
__device__ __forceinline__ float div_to_f32(double d, double s, double rs) {
  double q = d * rs;
  const uint32_t lo = (uint32_t)__double2loint(q) & 0x1FFFFFFFu;
  if (__builtin_expect(lo - 0x0FFFFFFCu < 8u, 0)) q = obs_ieee_div(d, s);
  return (float)q;
}

// NormalizeWrapper value of byte u at element e of the (y, x, c) frame, float64, as fp32
__device__ __forceinline__ float norm_value(uint32_t u, int mode, const double* __restrict__ mean, double stdv,
                                            double rstd, long long e) {
  if (mode == 2) return div_to_f32((double)u - mean[e], stdv, rstd);
  if (mode == 1) return div_to_f32((double)u, 255.0, 1.0 / 255.0);
  return (float)u;
}

// One block per frame (blocks walk frames): the frame's bytes are staged in LDS
// with coalesced dword loads, every pixel is normalised once (3 reciprocal products),
// the colour planes are written straight out and the grey value goes to LDS, from
// where the transposed mono plane is written (coalesced on the output side).
// Dynamic LDS: S*S*3 bytes (frame, rounded to dwords) + S*S floats (grey).
__global__ __launch_bounds__(OBS_THREADS) void obs_preprocess_kernel(
    const uint8_t* __restrict__ src, long long src_stride, int N, int S, int mode, const double* __restrict__ mean,
    double stdv, int mono, float* __restrict__ dst, long long dst_stride, int aligned) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int px = S * S, nb = px * 3, nw = (nb + 3) / 4;
  const double rstd = 1.0 / stdv;
  uint32_t* fw = reinterpret_cast<uint32_t*>(lds);
  float* gray = reinterpret_cast<float*>(lds + 4 * nw);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    const uint8_t* f = src + (size_t)n * src_stride;
    float* o = dst + (size_t)n * dst_stride;
    __syncthreads();   // the previous frame's LDS reads are done
    if (aligned) {
      const uint32_t* fs = reinterpret_cast<const uint32_t*>(f);
      for (int w = threadIdx.x; w < nw; w += OBS_THREADS) fw[w] = fs[w];   // nb % 4 == 0 when aligned
    } else {
      for (int b = threadIdx.x; b < nb; b += OBS_THREADS) lds[b] = f[b];
    }
    __syncthreads();
    for (int p = threadIdx.x; p < px; p += OBS_THREADS) {
      float v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        v[c] = norm_value(lds[3 * p + c], mode, mean, stdv, rstd, 3LL * p + c);
        o[(size_t)c * px + p] = v[c];
      }
      if (mono) {
        float gm = gray_f32(v[0], v[1], v[2]);
        if (mode == 0) gm = (float)(uint8_t)gm;   // mono.astype(uint8) when the frame is still u8
        gray[p] = gm;
      }
    }
    if (mono) {
      __syncthreads();
      for (int p = threadIdx.x; p < px; p += OBS_THREADS) {
        const int y = p / S, x = p - y * S;
        o[(size_t)3 * px + p] = gray[x * S + y];   // transposed pixel (see header)
      }
    }
  }
}

// Frame-walking form (S <= 84: at most PPT pixels per thread): each thread owns
// the same PPT pixels of every frame its block walks, so the float64 means of
// those pixels are loaded once per block into registers — the one-block-per-frame
// kernel above re-read the 169 KB mean array (84 x 84 x 3 float64) for every frame,
// more bytes than the frame itself moves.  The grey plane sits in LDS with row
// stride S + 1, so the transposed read (stride S + 1 between lanes) and the
// row-order write are both bank-conflict-free.
constexpr int PPT = 7, WALK_THREADS = 1024;
__global__ __launch_bounds__(WALK_THREADS) void obs_preprocess_walk_kernel(
    const uint8_t* __restrict__ src, long long src_stride, int N, int S, int mode, const double* __restrict__ mean,
    double stdv, int mono, float* __restrict__ dst, long long dst_stride, int aligned) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int px = S * S, nb = px * 3, nw = (nb + 3) / 4, tid = threadIdx.x;
  uint32_t* fw = reinterpret_cast<uint32_t*>(lds);
  float* gray = reinterpret_cast<float*>(lds + 4 * nw);   // [S][S + 1]
  const double rstd = 1.0 / stdv;
  double m[PPT][3];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int p = tid + WALK_THREADS * j;
#pragma unroll
    for (int c = 0; c < 3; ++c) m[j][c] = (mode == 2 && p < px) ? mean[3LL * p + c] : 0.0;
  }
  // aligned frames: the next frame's dwords (<= 6 per thread) are loaded into registers
  // while the current one is computed
  constexpr int DPT = (PPT * WALK_THREADS * 3 / 4 + WALK_THREADS - 1) / WALK_THREADS;
  uint32_t nx[DPT];
  auto fetch = [&](int n) {
    if (!aligned || n >= N) return;
    const uint32_t* fs = reinterpret_cast<const uint32_t*>(src + (size_t)n * src_stride);
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      const int w = tid + WALK_THREADS * i;
      if (w < nw) nx[i] = fs[w];
    }
  };
  fetch(blockIdx.x);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    const uint8_t* f = src + (size_t)n * src_stride;
    float* o = dst + (size_t)n * dst_stride;
    __syncthreads();   // the previous frame's LDS reads are done
    if (aligned) {
#pragma unroll
      for (int i = 0; i < DPT; ++i) {
        const int w = tid + WALK_THREADS * i;
        if (w < nw) fw[w] = nx[i];
      }
    } else {
      for (int b = tid; b < nb; b += WALK_THREADS) lds[b] = f[b];
    }
    __syncthreads();
    fetch(n + gridDim.x);
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int p = tid + WALK_THREADS * j;
      if (p < px) {
        float v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const uint32_t u = lds[3 * p + c];
          v[c] = mode == 2 ? div_to_f32((double)u - m[j][c], stdv, rstd)
                           : mode == 1 ? div_to_f32((double)u, 255.0, 1.0 / 255.0) : (float)u;
          o[(size_t)c * px + p] = v[c];
        }
        if (mono) {
          float gm = gray_f32(v[0], v[1], v[2]);
          if (mode == 0) gm = (float)(uint8_t)gm;
          const int y = p / S, x = p - y * S;
          gray[y * (S + 1) + x] = gm;
        }
      }
    }
    if (mono) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < PPT; ++j) {
        const int p = tid + WALK_THREADS * j;
        if (p < px) {
          const int y = p / S, x = p - y * S;
          o[(size_t)3 * px + p] = gray[x * (S + 1) + y];   // transposed pixel (see header)
        }
      }
    }
  }
}

// one thread per (env, element of one frame): walk the nstack slots upward
// (slot s reads slot s+1 before slot s+1 is written: no race, in place)
__global__ __launch_bounds__(OBS_THREADS) void frame_stack_kernel(float* __restrict__ stacked, int N, int nstack,
                                                                  long long fe, const float* __restrict__ obs,
                                                                  const uint8_t* __restrict__ done, int reset) {
  const long long total = (long long)N * fe;
  for (long long i = (long long)blockIdx.x * OBS_THREADS + threadIdx.x; i < total;
       i += (long long)gridDim.x * OBS_THREADS) {
    const int n = (int)(i / fe);
    const long long e = i - (long long)n * fe;
    float* st = stacked + (size_t)n * nstack * fe + e;
    const bool zero = reset || (done && done[n]);
    for (int s = 0; s + 1 < nstack; ++s) st[(size_t)s * fe] = zero ? 0.f : st[(size_t)(s + 1) * fe];
    st[(size_t)(nstack - 1) * fe] = obs[(size_t)n * fe + e];
  }
}

unsigned grid_for(long long total) {
  const long long b = (total + OBS_THREADS - 1) / OBS_THREADS;
  return (unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

PPO_API int ppo_obs_preprocess(const uint8_t* src, long long src_stride, int N, int S, int mode, const double* mean,
                               double stdv, int mono, float* dst, long long dst_stride, void* stream) {
  PPO_REQUIRE(N >= 0 && S > 0 && mode >= 0 && mode <= 2, "ppo_obs_preprocess: N=%d S=%d mode=%d", N, S, mode);
  PPO_REQUIRE(mode != 2 || (mean != nullptr && stdv != 0.0), "ppo_obs_preprocess: mode 2 needs mean and std != 0");
  PPO_REQUIRE(src_stride >= 3LL * S * S && dst_stride >= (3LL + (mono ? 1 : 0)) * S * S,
              "ppo_obs_preprocess: strides %lld / %lld too small for %dx%dx3", src_stride, dst_stride, S, S);
  const long long lds_bytes = 4LL * ((3LL * S * S + 3) / 4) + 4LL * S * S;
  PPO_REQUIRE(lds_bytes <= 160 * 1024, "ppo_obs_preprocess: %dx%d frames exceed the LDS (%lld B)", S, S, lds_bytes);
  if (N == 0) return 0;
  const int aligned = ((uintptr_t)src % 4 == 0) && (src_stride % 4 == 0) && ((3 * S * S) % 4 == 0);
  int slot;
  const bool prof = ppo_prof_begin("obs_preprocess", as_stream(stream), &slot);
  if (S * S <= PPT * WALK_THREADS) {   // frame-walking blocks, means in registers (one 16-wave block per CU)
    const long long walk_lds = 4LL * ((3LL * S * S + 3) / 4) + 4LL * S * (S + 1);
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
    const int grid = N < n_cu ? N : n_cu;
    obs_preprocess_walk_kernel<<<(unsigned)grid, WALK_THREADS, (size_t)walk_lds, as_stream(stream)>>>(
        src, src_stride, N, S, mode, mean, stdv, mono, dst, dst_stride, aligned);
  } else {
    obs_preprocess_kernel<<<(unsigned)(N < 4096 ? N : 4096), OBS_THREADS, (size_t)lds_bytes, as_stream(stream)>>>(
        src, src_stride, N, S, mode, mean, stdv, mono, dst, dst_stride, aligned);
  }
  // algorithmic bytes: 3 u8 in + (3 + mono) f32 out per pixel
  if (prof) ppo_prof_end(slot, as_stream(stream), (double)N * S * S * (3.0 + 4.0 * (3 + (mono ? 1 : 0))));
  PPO_LAUNCH_CHECK("obs_preprocess_kernel");
  return 0;
}

PPO_API int ppo_frame_stack(float* stacked, int N, int nstack, long long frame_elems, const float* obs,
                            const uint8_t* done, int reset, void* stream) {
  PPO_REQUIRE(N >= 0 && nstack >= 1 && frame_elems > 0, "ppo_frame_stack: N=%d nstack=%d frame=%lld", N, nstack,
              frame_elems);
  if (N == 0) return 0;
  frame_stack_kernel<<<grid_for((long long)N * frame_elems), OBS_THREADS, 0, as_stream(stream)>>>(
      stacked, N, nstack, frame_elems, obs, done, reset);
  PPO_LAUNCH_CHECK("frame_stack_kernel");
  return 0;
}
