// conv1 (model.py:177 Conv2d(4, 32, 8, stride 4) + ReLU) for the observation
// forms the reference's own env chain produces, as
// image-resident split-bf16 MFMA kernels:
//
//   SRC_F32  fp32 NCHW rows [4][84][84] — what T/run.py stores unchanged
//            (RolloutStorage's default fp32 obs plane, T/a2c_ppo_acktr/storage.py:12,
//            filled by VecPyTorch.step_wait, T/make_env.py:96-114);
//   SRC_RGB  raw u8 RGB frames [84][84][3] (21,168 B, a quarter of the fp32
//            plane's bytes per channel and 5.3x fewer bytes per frame), with the
//            env-side wrappers of the OTC v7 recipe (T/make_env.py:411-413) fused
//            into the operand loader:
//              NormalizeWrapper      x = fl32(((double)u - mean[y][x][c]) / std)
//                                    (T/sohojoe_wrappers.py:958-991; u/255 or raw
//                                    without a normaliser file: mean 0, std 255 / 1)
//              FrameStackMono(2)     channel 3 = cv2 RGB2GRAY of the normalised
//                                    frame, transposed: gray(x[:, x][y]) at (y, x)
//                                    (T/sohojoe_wrappers.py:563-638; obs.hip has
//                                    the standalone restatement)
//              TransposeImage + .float()   HWC -> CHW, fp32
//            The normalised values are bit-identical to ppo_obs_preprocess (the
//            reference chain): the float64 quotient is formed as d·(1/std) and,
//            when that lies within 4 units of the last double bit of an fp32
//            rounding midpoint (where it might round differently from the
//            IEEE quotient the reference computes), recomputed with the IEEE
//            division — so fl32(q) always equals fl32(fl64(d / std)).
//
// Arithmetic: both operands are fp32, split exactly into three
// bf16 parts (x = x_h + x_m + x_l); six part products (NP = 6, default; 9 = all,
// 1 = half-precision mode) per fp32 product on v_mfma_f32_16x16x32_bf16 with fp32
// accumulation — the same fp32 emulation as the conv2/conv3/fc kernels.
//
// Forward layout: one persistent block (8 waves) per CU walks images; an image
// is 5 parts of 4 output rows (80 output pixels, 20 input rows).  A part's input
// rows sit in LDS as the three bf16 planes [plane][c][20][84] (40,320 B; two
// stages).  Wave w owns output channels 16 (w & 1) + [0, 16) and input channel
// c = w >> 1 (K = 64 of 256: two k-steps), for all five 16-pixel row tiles of
// the part, with its 2 x 3 weight fragments in registers (24 VGPRs).  The four
// channel partials meet in LDS and every thread finishes (pixel, channel) pairs
// in a fixed order: Σ_c, + bias, ReLU, coalesced 128-B row stores, and the ReLU
// mask bits by ballot.  The next part is staged (split VALU + LDS writes) by
// every wave ahead of its MFMAs; its raw data is one part ahead in registers
// (SRC_F32) or the whole u8 frame sits in LDS (SRC_RGB, 21 KB, loaded into
// registers during the previous image).
#include "igemm.h"
#include "igemm_x9.h"

namespace {

constexpr int IMG = 84, IMG2 = IMG * IMG, RGBB = IMG2 * 3;   // RGB frame bytes (21,168)
constexpr int NPART = 5, PROWS = 20;
// forward stage: a part's 20 input rows per channel, the channel blocks padded to
// 1,728 elements (864 dwords = 32 mod 64 banks) so that the lane groups reading
// channels c and c + 1 of one k-step hit disjoint bank halves
constexpr int CSTR = PROWS * IMG + 48, PLANE = 4 * CSTR;   // bf16 elements per plane of a part (6,912)
constexpr int PSTR = 36;   // LDS row stride (floats) of the channel partials: 4 px apart -> 16 banks apart
enum { SRC_F32 = 0, SRC_RGB = 1 };

// fl32(fl64((u - m) / s)) bit-exactly (see header): q = d·(1/s); the 29 bits a
// rounding to fp32 drops decide; within 4 of the midpoint pattern, take d / s
__device__ __attribute__((noinline)) double ieee_div(double d, double s) { return d / s; }   // the rare path
__device__ __forceinline__ float norm_u8(uint32_t u, float m, double s, double rs) {
  const double d = (double)u - (double)m;   // exact: u integer, m fp32
  double q = d * rs;
  const uint32_t lo = (uint32_t)__double2loint(q) & 0x1FFFFFFFu;
  if (__builtin_expect(lo - 0x0FFFFFFCu < 8u, 0)) q = ieee_div(d, s);   // near a midpoint: the IEEE quotient
  return (float)q;
}
// cv2 RGB2GRAY on fp32 (R·0.299 + G·0.587) + B·0.114, one rounding per op (no
// FMA contraction: __fmul_rn / __fadd_rn are plain operators hipcc would fuse);
// u8: FrameStackMono stores the grey plane in the frame's dtype — still u8 when
// no normaliser ran (raw mode) — i.e. truncated (.astype(np.uint8))
__device__ __forceinline__ float gray3(float r, float g, float b, bool u8) {
#pragma clang fp contract(off)
  const float v = (r * 0.299f + g * 0.587f) + b * 0.114f;
  return u8 ? (float)(uint8_t)v : v;
}


// 4 fp32 -> the three bf16 planes' 4-element pieces (uint2 each), each part the
// RNE of the remaining residual (v_cvt_pk_bf16_f32); NPL 1: hi only
template <int NPL>
__device__ __forceinline__ void split4(const f32x4& v, uint2 (&o)[3]) {
  uint32_t w[3][2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    f32x2 x = f32x2{v[2 * p], v[2 * p + 1]};
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl) {
      const bf16x2 b = __builtin_convertvector(x, bf16x2);
      w[pl][p] = __builtin_bit_cast(uint32_t, b);
      if (pl + 1 < NPL) x = x - f32x2{(float)b[0], (float)b[1]};
    }
  }
#pragma unroll
  for (int pl = 0; pl < NPL; ++pl) o[pl] = uint2{w[pl][0], w[pl][1]};
}

// c += Σ_{(i,j) in the product set} a_i · w_j, smallest first
template <int NP>
__device__ __forceinline__ f32x4 mma_set(const bf16x8 (&a)[3], const bf16x8 (&wq)[3], f32x4 c) {
  if constexpr (NP == 1) return mma(a[0], wq[0], c);
  if constexpr (NP == 9) {
    c = mma(a[2], wq[2], c);
    c = mma(a[2], wq[1], c);
    c = mma(a[1], wq[2], c);
  }
  c = mma(a[1], wq[1], c);
  c = mma(a[2], wq[0], c);
  c = mma(a[0], wq[2], c);
  c = mma(a[1], wq[0], c);
  c = mma(a[0], wq[1], c);
  return mma(a[0], wq[0], c);
}

// means of normalisation item t of part p (see rgb_item): 12 fp32 values
__device__ __forceinline__ void rgb_means(int t, int p, const float* __restrict__ mean, f32x4 (&m)[3]) {
  if (t < 420) {
    const int yl = t / 21, q = t - 21 * yl;
    const f32x4* mp = reinterpret_cast<const f32x4*>(mean + ((16 * p + yl) * IMG + 4 * q) * 3);
    m[0] = mp[0];
    m[1] = mp[1];
    m[2] = mp[2];
  } else if (t < 840) {
    const int yl = (t - 420) / 21, q = (t - 420) - 21 * yl, y = 16 * p + yl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float* mp = mean + ((4 * q + j) * IMG + y) * 3;
      m[0][j] = mp[0];
      m[1][j] = mp[1];
      m[2][j] = mp[2];
    }
  }
}

// byte i (0..11) of three packed dwords / mean i of three float4 (i compile-time after unrolling)
__device__ __forceinline__ uint32_t byte_of(uint32_t w0, uint32_t w1, uint32_t w2, int i) {
  const uint32_t w = i < 4 ? w0 : (i < 8 ? w1 : w2);
  return (w >> (8 * (i & 3))) & 255u;
}
__device__ __forceinline__ float mean_of(const f32x4 (&m)[3], int i) {
  const f32x4 v = i < 4 ? m[0] : (i < 8 ? m[1] : m[2]);
  return v[i & 3];
}

// One normalisation item of part p (NormalizeWrapper + FrameStackMono(2) decode of
// the u8 frame in LDS): t < 420 colour quad (yl, q) -> channels 0..2 at
// (16p + yl, 4q .. 4q + 3); 420 <= t < 840 grey quad -> channel 3 at the same
// positions, gray of the transposed pixels (4q + j, 16p + yl).  The 4 values go
// to `dst` either split into NPL bf16 planes (plane stride pstride, channel stride
// cstride elements; NPL = 0: as fp32 into a float scratch with channel stride cstride).
template <int NPL, typename T>
__device__ __forceinline__ void rgb_item(int t, int p, const uint8_t* __restrict__ R8, bool has_mean,
                                         const f32x4 (&m)[3], double s, double rs, T* __restrict__ dst, int cstride,
                                         int pstride, int rstride = IMG) {
  if (t < 420) {
    const int yl = t / 21, q = t - 21 * yl;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(R8 + ((16 * p + yl) * IMG + 4 * q) * 3);
    const uint32_t w0 = s32[0], w1 = s32[1], w2 = s32[2];   // 4 px x RGB
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = norm_u8(byte_of(w0, w1, w2, 3 * j + c), has_mean ? mean_of(m, 3 * j + c) : 0.f, s, rs);
      const int off = c * cstride + yl * rstride + 4 * q;
      if constexpr (NPL == 0) {
        *reinterpret_cast<f32x4*>(dst + off) = v;
      } else {
        uint2 o[3];
        split4<NPL>(v, o);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) *reinterpret_cast<uint2*>(dst + pl * pstride + off) = o[pl];
      }
    }
  } else if (t < 840) {
    const int yl = (t - 420) / 21, q = (t - 420) - 21 * yl, y = 16 * p + yl;
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint8_t* px = R8 + ((4 * q + j) * IMG + y) * 3;
      v[j] = gray3(norm_u8(px[0], has_mean ? m[0][j] : 0.f, s, rs), norm_u8(px[1], has_mean ? m[1][j] : 0.f, s, rs),
                   norm_u8(px[2], has_mean ? m[2][j] : 0.f, s, rs), !has_mean && s == 1.0);
    }
    const int off = 3 * cstride + yl * rstride + 4 * q;
    if constexpr (NPL == 0) {
      *reinterpret_cast<f32x4*>(dst + off) = v;
    } else {
      uint2 o[3];
      split4<NPL>(v, o);
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) *reinterpret_cast<uint2*>(dst + pl * pstride + off) = o[pl];
    }
  }
}

template <int SRC, bool MASK, int NP>
__global__ __launch_bounds__(512) void conv1_fwd_x6_kernel(const void* __restrict__ obs, const int64_t* __restrict__ idx,
                                                           long long row0, int B, const float* __restrict__ mean,
                                                           double stdv, double rstd, const float* __restrict__ w,
                                                           const float* __restrict__ bias, float* __restrict__ out,
                                                           uint32_t* __restrict__ mbits, int dbg) {
  // dbg (timing anatomy only, wrong results): 1 skips the MFMAs, 2 the staging,
  // 4 the global loads, 8 the partial sums + epilogue, 16 the stagger
  const bool no_mma = dbg & 1, no_put = dbg & 2, no_ld = dbg & 4, no_epi = dbg & 8;
  constexpr int NPL = NP == 1 ? 1 : 3;   // planes staged
  constexpr int NPW = NP == 1 ? 1 : 3;   // weight parts
  __shared__ __attribute__((aligned(16))) uint16_t X[2][NPL][PLANE];
  __shared__ __attribute__((aligned(16))) float P[4][80 * PSTR];
  __shared__ __attribute__((aligned(16))) uint8_t R8[SRC == SRC_RGB ? RGBB + 16 : 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, kq = wave >> 1, i16 = lane & 15, g = lane >> 4;
  const bool late = wave >= 4 && !(dbg & 16);   // per SIMD one wave stages before its MFMAs, one after
  const int G = gridDim.x;
  const int nimg = (int)blockIdx.x < B ? (B - 1 - (int)blockIdx.x) / G + 1 : 0, nit = NPART * nimg;
  // k order: k-step = one kernel row ky (32 k = 4 channels x 8 kx), lane group g =
  // channel g; wave (ct, kq) takes ky = 2 kq + si.  Weight fragments B[k][n] = W[n][k]
  bf16x8 wf[2][3];
#pragma unroll
  for (int si = 0; si < 2; ++si) {
    const float* wp = w + (size_t)(16 * ct + i16) * 256 + 64 * g + 8 * (2 * kq + si);
    uint32_t h[8], m[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (NPW == 3) split_bf16x3(wp[j], h[j], m[j], l[j]);
      else h[j] = bf16_rne_bits(wp[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wf[si][0][j] = __builtin_bit_cast(__bf16, (uint16_t)h[j]);
      if constexpr (NPW == 3) {
        wf[si][1][j] = __builtin_bit_cast(__bf16, (uint16_t)m[j]);
        wf[si][2][j] = __builtin_bit_cast(__bf16, (uint16_t)l[j]);
      }
    }
  }
  const float bv = bias[tid & 31];
  wait_vm0();

  // ---------------- raw data: SRC_F32 one part ahead in registers
  f32x4 xr[4];
  auto fetch_f32 = [&](int it) __attribute__((always_inline)) {
    if (it >= nit || no_ld) return;
    const int k = it / NPART, p = it - NPART * k;
    const float* base = reinterpret_cast<const float*>(obs) + obs_row(idx, row0, (int)blockIdx.x + k * G) * (4LL * IMG2) +
                        p * 16 * IMG;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = tid + 512 * j;
      if (f < 1680) {
        const int c = f / 420, rem = f - 420 * c, yl = rem / 21, q = rem - 21 * yl;
        xr[j] = *reinterpret_cast<const f32x4*>(base + c * IMG2 + yl * IMG + 4 * q);
      }
    }
  };
  auto put_f32 = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = tid + 512 * j;
      if (f < 1680) {
        const int c = f / 420, rem = f - 420 * c, yl = rem / 21, q = rem - 21 * yl;
        uint2 o[3];
        split4<NPL>(xr[j], o);
        const int off = c * CSTR + yl * IMG + 4 * q;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) *reinterpret_cast<uint2*>(&X[st][pl][off]) = o[pl];
      }
    }
  };
  // ---------------- SRC_RGB: the frame in LDS, the next frame in registers; means one part ahead
  uint4 fr[3];
  auto fetch_frame = [&](int k) __attribute__((always_inline)) {
    if (k >= nimg) return;
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(obs) +
                                                      obs_row(idx, row0, (int)blockIdx.x + k * G) * (long long)RGBB);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = tid + 512 * j;
      if (c < RGBB / 16) fr[j] = src[c];
    }
  };
  auto store_frame = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = tid + 512 * j;
      if (c < RGBB / 16) *reinterpret_cast<uint4*>(R8 + 16 * c) = fr[j];
    }
  };
  // item t of a part: t < 420 colour quad (yl, q): pixels (16p + yl, 4q + j), all three
  // channels; 420 <= t < 840 grey quad: grey at (16p + yl, 4q + j) = gray of pixel
  // (4q + j, 16p + yl) (the transposed mono plane).  Thread tid: items tid, tid + 512.
  f32x4 mA[3], mB[3];   // means of the thread's two items of the next part
  auto fetch_means = [&](int it) __attribute__((always_inline)) {
    if (it >= nit || mean == nullptr || no_ld) return;
    const int p = it % NPART;
    rgb_means(tid, p, mean, mA);
    rgb_means(tid + 512, p, mean, mB);
  };
  auto put_rgb = [&](int it, int st) __attribute__((always_inline)) {
    const int p = it % NPART;
    rgb_item<NPL>(tid, p, R8, mean != nullptr, mA, stdv, rstd, &X[st][0][0], CSTR, PLANE);
    rgb_item<NPL>(tid + 512, p, R8, mean != nullptr, mB, stdv, rstd, &X[st][0][0], CSTR, PLANE);
  };

  // ---------------- compute: wave (ct, kq), five row tiles, two k-steps (ky = 2 kq + si)
  int pix[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int px = 16 * t + i16, oyl = px / 20, ox = px - 20 * oyl;
    pix[t] = g * CSTR + (4 * oyl + 2 * kq) * IMG + 4 * ox;   // + IMG si
  }
  auto compute = [&](int st) __attribute__((always_inline)) {
    f32x4 acc[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = zero4();
    if (!no_mma) {
#pragma unroll
      for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          bf16x8 a[3];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) {
            const uint2* p2 = reinterpret_cast<const uint2*>(&X[st][pl][pix[t] + IMG * si]);
            const uint2 lo = p2[0], hi = p2[1];
            a[pl] = __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y});
          }
          acc[t] = mma_set<NP>(a, wf[si], acc[t]);
        }
    }
    if (no_epi) return;
    // this wave's partial over its two kernel rows: acc[t][r] = out[px 16 t + 4 g + r][co 16 ct + i16]
    float* Pc = P[kq];
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) Pc[(16 * t + 4 * g + r) * PSTR + 16 * ct + i16] = acc[t][r];
  };
  auto epilogue = [&](int it) __attribute__((always_inline)) {
    if (no_epi) return;
    const int k = it / NPART, p = it - NPART * k, b = (int)blockIdx.x + k * G;
    const int co = tid & 31;
    float* o = out + (size_t)b * (400 * 32) + (size_t)(80 * p) * 32;
#pragma unroll
    for (int e = 0; e < 5; ++e) {
      const int px = (tid >> 5) + 16 * e;
      const int a = px * PSTR + co;
      const float v = fmaxf(((P[0][a] + P[1][a]) + (P[2][a] + P[3][a])) + bv, 0.f);
      o[px * 32 + co] = v;
      if constexpr (MASK) {
        const uint64_t bal = __builtin_amdgcn_ballot_w64(v > 0.f);
        if ((lane & 31) == 0) mbits[(size_t)b * 400 + 80 * p + px] = (uint32_t)(bal >> (lane & 32));
      }
    }
  };

  // ---------------- pipeline: stage it + 1 while computing it
  auto put = [&](int it, int st) __attribute__((always_inline)) {
    if (no_put) return;
    if constexpr (SRC == SRC_F32) put_f32(st);
    else put_rgb(it, st);
  };
  auto prefetch = [&](int it) __attribute__((always_inline)) {   // raw data / means of item it into registers
    if constexpr (SRC == SRC_F32) fetch_f32(it);
    else fetch_means(it);
  };
  if (nit > 0) {
    if constexpr (SRC == SRC_RGB) {
      fetch_frame(0);
      store_frame();
      fetch_frame(1);
      lds_barrier();
    }
    prefetch(0);
    put(0, 0);
    prefetch(1);
  }
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const int st = it & 1;
    if (it + 1 < nit) {
      if constexpr (SRC == SRC_RGB) {
        if ((it + 1) % NPART == 0) {   // the next item starts a new frame: every put of this one is done
          store_frame();
          fetch_frame((it + 1) / NPART + 1);
          lds_barrier();
        }
      }
      if (!late) {
        put(it + 1, st ^ 1);
        prefetch(it + 2);
      }
    }
    compute(st);
    if (late && it + 1 < nit) {
      put(it + 1, st ^ 1);
      prefetch(it + 2);
    }
    lds_barrier();   // partials complete; stage st ^ 1 complete
    epilogue(it);
    lds_barrier();   // partials consumed before the next item writes them
  }
}


// Forward, full-K form (fp32 rows; the RGB decode takes the K-split kernel
// above): 10 waves, wave w = (column tile w & 1, row tile w >> 1) of the part
// computes its 16 x 16 output tile over all 256 k (8 k-steps, one kernel row
// each) with all 8 x 3 weight fragments resident (96 VGPRs), so no partial sums
// cross waves: the epilogue (bias, ReLU, stores, mask bits) follows the wave's
// own MFMAs and one barrier per part remains.  The price is the SIMD balance
// (3, 3, 2, 2 waves): at most 5/6 of the MFMA rate.
template <int SRC, bool MASK, int NP>
__global__ __launch_bounds__(640) void conv1_fwd_x6w_kernel(const void* __restrict__ obs, const int64_t* __restrict__ idx,
                                                            long long row0, int B, const float* __restrict__ mean,
                                                            double stdv, double rstd, const float* __restrict__ w,
                                                            const float* __restrict__ bias, float* __restrict__ out,
                                                            uint32_t* __restrict__ mbits, int dbg) {
  const bool no_mma = dbg & 1, no_put = dbg & 2, no_ld = dbg & 4, no_epi = dbg & 8;
  constexpr int NTH = 640;
  constexpr int NPL = NP == 1 ? 1 : 3;
  constexpr int NPW = NP == 1 ? 1 : 3;
  __shared__ __attribute__((aligned(16))) uint16_t X[2][NPL][PLANE];
  __shared__ __attribute__((aligned(16))) uint8_t R8[SRC == SRC_RGB ? RGBB + 16 : 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, rt = wave >> 1, i16 = lane & 15, g = lane >> 4;
  const bool late = ((wave >> 2) & 1) != 0 && !(dbg & 16);
  const int G = gridDim.x;
  const int nimg = (int)blockIdx.x < B ? (B - 1 - (int)blockIdx.x) / G + 1 : 0, nit = NPART * nimg;
  const int col = 16 * ct + i16;
  // k-step ky: 32 k = 4 channels (lane group g) x 8 kx; B[k][n] = W[n][g][ky][j]
  bf16x8 wf[8][3];
#pragma unroll
  for (int ky = 0; ky < 8; ++ky) {
    const float* wp = w + (size_t)col * 256 + 64 * g + 8 * ky;
    uint32_t h[8], m[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (NPW == 3) split_bf16x3(wp[j], h[j], m[j], l[j]);
      else h[j] = bf16_rne_bits(wp[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wf[ky][0][j] = __builtin_bit_cast(__bf16, (uint16_t)h[j]);
      if constexpr (NPW == 3) {
        wf[ky][1][j] = __builtin_bit_cast(__bf16, (uint16_t)m[j]);
        wf[ky][2][j] = __builtin_bit_cast(__bf16, (uint16_t)l[j]);
      }
    }
  }
  const float bv = bias[col];
  wait_vm0();

  f32x4 xr[3];
  auto fetch_f32 = [&](int it) __attribute__((always_inline)) {
    if (it >= nit || no_ld) return;
    const int k = it / NPART, p = it - NPART * k;
    const float* base = reinterpret_cast<const float*>(obs) + obs_row(idx, row0, (int)blockIdx.x + k * G) * (4LL * IMG2) +
                        p * 16 * IMG;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int f = tid + NTH * j;
      if (f < 1680) {
        const int c = f / 420, rem = f - 420 * c, yl = rem / 21, q = rem - 21 * yl;
        xr[j] = *reinterpret_cast<const f32x4*>(base + c * IMG2 + yl * IMG + 4 * q);
      }
    }
  };
  auto put_f32 = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int f = tid + NTH * j;
      if (f < 1680) {
        const int c = f / 420, rem = f - 420 * c, yl = rem / 21, q = rem - 21 * yl;
        uint2 o[3];
        split4<NPL>(xr[j], o);
        const int off = c * CSTR + yl * IMG + 4 * q;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) *reinterpret_cast<uint2*>(&X[st][pl][off]) = o[pl];
      }
    }
  };
  uint4 fr[3];
  auto fetch_frame = [&](int k) __attribute__((always_inline)) {
    if (k >= nimg || no_ld) return;
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(obs) +
                                                      obs_row(idx, row0, (int)blockIdx.x + k * G) * (long long)RGBB);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = tid + NTH * j;
      if (c < RGBB / 16) fr[j] = src[c];
    }
  };
  auto store_frame = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int c = tid + NTH * j;
      if (c < RGBB / 16) *reinterpret_cast<uint4*>(R8 + 16 * c) = fr[j];
    }
  };
  f32x4 mA[3], mB[3];   // means of the thread's items tid, tid + 640 of the next part
  auto fetch_means = [&](int it) __attribute__((always_inline)) {
    if (it >= nit || mean == nullptr || no_ld) return;
    const int p = it % NPART;
    rgb_means(tid, p, mean, mA);
    rgb_means(tid + NTH, p, mean, mB);
  };
  auto put = [&](int it, int st) __attribute__((always_inline)) {
    if (no_put) return;
    if constexpr (SRC == SRC_F32) {
      put_f32(st);
    } else {
      const int p = it % NPART;
      rgb_item<NPL>(tid, p, R8, mean != nullptr, mA, stdv, rstd, &X[st][0][0], CSTR, PLANE);
      rgb_item<NPL>(tid + NTH, p, R8, mean != nullptr, mB, stdv, rstd, &X[st][0][0], CSTR, PLANE);
    }
  };
  auto prefetch = [&](int it) __attribute__((always_inline)) {
    if constexpr (SRC == SRC_F32) fetch_f32(it);
    else fetch_means(it);
  };
  // the lane's A row: output pixel 16 rt + i16 of the part; k-step ky adds ky rows
  const int px = 16 * rt + i16, oyl = px / 20, ox = px - 20 * oyl;
  const int pix = g * CSTR + 4 * oyl * IMG + 4 * ox;
  auto compute = [&](int it) __attribute__((always_inline)) {
    const int st = it & 1;
    f32x4 acc = zero4();
    if (!no_mma) {
#pragma unroll
      for (int ky = 0; ky < 8; ++ky) {
        bf16x8 a[3];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const uint2* p2 = reinterpret_cast<const uint2*>(&X[st][pl][pix + IMG * ky]);
          const uint2 lo = p2[0], hi = p2[1];
          a[pl] = __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y});
        }
        acc = mma_set<NP>(a, wf[ky], acc);
      }
    }
    if (no_epi) return;
    const int k = it / NPART, p = it - NPART * k, b = (int)blockIdx.x + k * G;
    float* o = out + ((size_t)b * 400 + 80 * p + 16 * rt) * 32 + col;
    uint64_t bal[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = fmaxf(acc[r] + bv, 0.f);
      o[(4 * g + r) * 32] = v;
      if constexpr (MASK) bal[r] = __builtin_amdgcn_ballot_w64(v > 0.f);
    }
    if constexpr (MASK) {   // lane (g, i16) of ballot r: pixel 4 g + r, channel col; lane j < 16 stores pixel j's 16 bits
      if (lane < 16) {
        const int r = lane & 3, gg = lane >> 2;
        const uint64_t bsel = r == 0 ? bal[0] : r == 1 ? bal[1] : r == 2 ? bal[2] : bal[3];
        reinterpret_cast<uint16_t*>(mbits)[((size_t)b * 400 + 80 * p + 16 * rt + lane) * 2 + ct] =
            (uint16_t)(bsel >> (16 * gg));
      }
    }
  };

  if (nit > 0) {
    if constexpr (SRC == SRC_RGB) {
      fetch_frame(0);
      store_frame();
      fetch_frame(1);
      lds_barrier();
    }
    prefetch(0);
    put(0, 0);
    prefetch(1);
  }
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const bool more = it + 1 < nit;
    if constexpr (SRC == SRC_RGB) {
      if (more && (it + 1) % NPART == 0) {
        store_frame();
        fetch_frame((it + 1) / NPART + 1);
        lds_barrier();
      }
    }
    if (more && !late) {
      put(it + 1, (it + 1) & 1);
      prefetch(it + 2);
    }
    compute(it);
    if (more && late) {
      put(it + 1, (it + 1) & 1);
      prefetch(it + 2);
    }
    lds_barrier();
  }
}

// ---------------------------------------------------------------------------
// Weight gradient: dW[co][(c, ky, kx)] = Σ_px dz1[px][co] · x[c][4oy+ky][4ox+kx]
// (the backward of model.py:177 in loss.backward(), algo/ppo.py:80-81), for the
// same two sources.  M = 32 output channels, N = 256 columns, K = pixels, on
// v_mfma_f32_32x32x16_bf16, both operands split three ways (NP part products).
// An image is 5 parts of 4 output rows (80 px = 5 k-steps).  Per part, double
// buffered:
//   S  the part's 20 input rows of all 4 channels, split once into the three
//      bf16 planes [plane][c][20][96] — SRC_F32 from registers (one part ahead),
//      SRC_RGB normalised from the u8 frame in LDS (the exact decode, the grey
//      plane transposed);
//   D  dz of the part split into three bf16 planes [32 co][88] (A fragments,
//      ds_read_b128).
// The im2col B fragment (8 pixels x 32 columns (ky, kx) of one channel) comes
// straight from S with two ds_read_b64_tr_b16 per plane: in each 16-lane group,
// lane 4q + p addresses pixel q's 4 consecutive kx (4 (p & 1) .. +3) of kernel
// row 2 (lane group & 1) + (p >> 1) — 8 contiguous, 8-B aligned bytes of an
// image row — and lane i receives column i of the 4 pixels.  No expanded copy,
// no VALU on the image operand.  Row stride 96 (48 dwords): the four kernel rows
// of one read sit 0 / 48 / 32 / 16 banks apart, conflict-free.
// 16 waves: wave w takes the column tiles of channel w & 3 (both kernel-row
// halves: one dz fragment feeds two tiles) and the k-steps ≡ w >> 2 (mod 4) of
// the part sequence; the four k-group partials are summed in a fixed order at
// the end.  Per SIMD one wave stages the next part before its MFMAs, one after.
// Output: the split-K slab [Z][32][256] and bias partials [Z][32] (fp32 values:
// reduce with scale 1).
constexpr int SRS = 96, SCH = PROWS * SRS, SPL = 4 * SCH;   // bf16 S: row / channel / plane strides
constexpr int DZS = 88, DZPL = 32 * DZS;                    // bf16 per dz plane
constexpr int WMAXIMG = 512;

template <int NP>
__device__ __forceinline__ f32x16 mma32_set(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
#define M32(x, y) c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[x], b[y], c, 0, 0, 0)
  if constexpr (NP == 1) {
    M32(0, 0);
    return c;
  }
  if constexpr (NP == 9) {
    M32(2, 2);
    M32(2, 1);
    M32(1, 2);
  }
  M32(1, 1);
  M32(2, 0);
  M32(0, 2);
  M32(1, 0);
  M32(0, 1);
  M32(0, 0);
#undef M32
  return c;
}

template <int SRC, int NP>
__global__ __launch_bounds__(1024) void conv1_wgrad_x6_kernel(const float* __restrict__ dz1,
                                                              const void* __restrict__ obs,
                                                              const int64_t* __restrict__ idx, long long row0, int B,
                                                              const float* __restrict__ mean, double stdv, double rstd,
                                                              float* __restrict__ slab, float* __restrict__ slab_bias,
                                                              int dbg) {
  // dbg (timing anatomy only, wrong results): 1 skips the MFMAs, 2 the staging,
  // 4 the global loads, 16 the stagger
  const bool no_mma = dbg & 1, no_put = dbg & 2, no_ld = dbg & 4;
  constexpr int NPL = NP == 1 ? 1 : 3;                  // dz and image planes
  __shared__ __attribute__((aligned(16))) uint16_t S[2][3][SPL];   // 3 planes even at NPL 1: the k-group scratch
  __shared__ __attribute__((aligned(16))) uint16_t D[2][NPL][DZPL];
  __shared__ __attribute__((aligned(16))) uint8_t R8[SRC == SRC_RGB ? RGBB + 16 : 16];
  __shared__ int rowtab[WMAXIMG];
  __shared__ float bred[320];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int wc = wave & 3, kg = wave >> 2;   // channel (tiles 2 wc, 2 wc + 1), k-group
  const bool late = (wave & 4) != 0 && !(dbg & 16);
  const int G = gridDim.x;
  const int nimg = (int)blockIdx.x < B ? (B - 1 - (int)blockIdx.x) / G + 1 : 0;
  const int nit = NPART * nimg;
  for (int k = tid; k < nimg; k += 1024) rowtab[k] = (int)obs_row(idx, row0, (int)blockIdx.x + k * G);
  // tr-read lane roles: 16-lane group lg = lane >> 4 (columns 16 (lg & 1) .., k half
  // lg >> 1), lane 4 tq + tp of it: pixel tq of the read, kernel row
  // 2 (lg & 1) + (tp >> 1) of the tile, kx 4 (tp & 1) .. +3
  const int lg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int tcol = wc * SCH + (2 * (lg & 1) + (tp >> 1)) * SRS + 4 * (tp & 1);
  const int aoff = l32 * DZS + 8 * h;   // + 16 ls
  const bool d_on = tid >= 512 && tid < 832;
  const int dit = d_on ? tid - 512 : 0, dco = dit & 31, doc = dit >> 5;
  float bacc = 0.f;
  __syncthreads();   // rowtab

  // ---------------- raw data in registers, one part ahead
  f32x4 xr[2];    // SRC_F32: the part's rows, 1,680 float4
  float dv[8];    // dz item: 8 pixels of one channel
  auto fetch = [&](int it) __attribute__((always_inline)) {
    if (it >= nit || no_ld) return;
    const int k = it / NPART, p = it - NPART * k;
    if constexpr (SRC == SRC_F32) {
      const float* base = reinterpret_cast<const float*>(obs) + (long long)rowtab[k] * (4LL * IMG2) + p * 16 * IMG;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int f = tid + 1024 * j;
        if (f < 1680) {
          const int c = f / 420, rem = f - 420 * c, yl = rem / 21, q = rem - 21 * yl;
          xr[j] = *reinterpret_cast<const f32x4*>(base + c * IMG2 + yl * IMG + 4 * q);
        }
      }
    }
    if (d_on) {
      const float* src = dz1 + ((size_t)((int)blockIdx.x + k * G) * 400 + 80 * p + 8 * doc) * 32 + dco;
#pragma unroll
      for (int q = 0; q < 8; ++q) dv[q] = src[32 * q];
    }
  };
  // ---------------- SRC_RGB: frame in LDS (next one in registers), means one part ahead
  uint4 fr[2];
  f32x4 mr[3];
  auto fetch_frame = [&](int k) __attribute__((always_inline)) {
    if (k >= nimg || no_ld) return;
    const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(obs) +
                                                      (long long)rowtab[k] * RGBB);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 1024 * j;
      if (c < RGBB / 16) fr[j] = src[c];
    }
  };
  auto store_frame = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 1024 * j;
      if (c < RGBB / 16) *reinterpret_cast<uint4*>(R8 + 16 * c) = fr[j];
    }
  };
  auto fetch_means = [&](int it) __attribute__((always_inline)) {
    if (it < nit && mean != nullptr && !no_ld) rgb_means(tid, it % NPART, mean, mr);
  };
  // ---------------- put part it into stage it & 1: S planes and the dz planes
  auto put = [&](int it) __attribute__((always_inline)) {
    if (no_put) return;
    const int st = it & 1;
    if constexpr (SRC == SRC_F32) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int f = tid + 1024 * j;
        if (f < 1680) {
          const int c = f / 420, rem = f - 420 * c, yl = rem / 21, q = rem - 21 * yl;
          uint2 o[3];
          split4<NPL>(xr[j], o);
          const int off = c * SCH + yl * SRS + 4 * q;
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) *reinterpret_cast<uint2*>(&S[st][pl][off]) = o[pl];
        }
      }
    } else {
      rgb_item<NPL>(tid, it % NPART, R8, mean != nullptr, mr, stdv, rstd, &S[st][0][0], SCH, SPL, SRS);
    }
    if (d_on) {
      Frag3 fr3;
      split8(f32x4{dv[0], dv[1], dv[2], dv[3]}, f32x4{dv[4], dv[5], dv[6], dv[7]}, fr3, NPL == 1);
      uint16_t* d0 = &D[st][0][dco * DZS + 8 * doc];
      *reinterpret_cast<bf16x8*>(d0) = fr3.h;
      if constexpr (NPL == 3) {
        *reinterpret_cast<bf16x8*>(d0 + DZPL) = fr3.m;
        *reinterpret_cast<bf16x8*>(d0 + 2 * DZPL) = fr3.l;
      }
      bacc += ((dv[0] + dv[1]) + (dv[2] + dv[3])) + ((dv[4] + dv[5]) + (dv[6] + dv[7]));
    }
  };
  auto prefetch = [&](int it) __attribute__((always_inline)) {
    fetch(it);
    if constexpr (SRC == SRC_RGB) fetch_means(it);
  };

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  auto compute = [&](int it) __attribute__((always_inline)) {
    if (no_mma) return;
    const int st = it & 1;
    // the wave's k-steps of this part: ls ≡ kg - 5 it (mod 4), at most two
    const int ls0 = (kg - 5 * it) & 3;
#pragma unroll 1
    for (int ls = ls0; ls < 5; ls += 4) {
      bf16x8 a[3];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) a[pl] = *reinterpret_cast<const bf16x8*>(&D[st][pl][aoff + 16 * ls]);
      int ro[2];   // S offset of this lane's tr-read row: pixel 16 ls + 8 (lg >> 1) + 4 rd + tq
#pragma unroll
      for (int rd = 0; rd < 2; ++rd) {
        const int px = 16 * ls + 8 * (lg >> 1) + 4 * rd + tq, oyl = px / 20, ox = px - 20 * oyl;
        ro[rd] = tcol + 4 * oyl * SRS + 4 * ox;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {   // kernel-row half t: ky = 4 t + (column >> 3)
        bf16x8 b[3];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          s16x4 v[2];
#pragma unroll
          for (int rd = 0; rd < 2; ++rd)
            v[rd] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(&S[st][pl][ro[rd] + 4 * t * SRS]));
          b[pl] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7));
        }
        acc[t] = mma32_set<NP>(a, b, acc[t]);
      }
    }
  };

  // ---------------- pipeline
  if (nit > 0) {
    if constexpr (SRC == SRC_RGB) {
      fetch_frame(0);
      store_frame();
      fetch_frame(1);
      lds_barrier();   // frame 0
    }
    prefetch(0);
    put(0);
    prefetch(1);
  }
  __syncthreads();
  for (int it = 0; it < nit; ++it) {
    const bool more = it + 1 < nit;
    if constexpr (SRC == SRC_RGB) {
      if (more && (it + 1) % NPART == 0) {   // part it + 1 opens a new frame: every put of this one is done
        store_frame();
        fetch_frame((it + 1) / NPART + 1);
        lds_barrier();
      }
    }
    if (more && !late) {
      put(it + 1);
      prefetch(it + 2);
    }
    compute(it);
    if (more && late) {
      put(it + 1);
      prefetch(it + 2);
    }
    lds_barrier();
  }
  // k-group partials -> (k0 + k2) + (k1 + k3) in three rounds through one 32-KB
  // slot of the S space (free now): k1 += k3; k0 += k2; k0 += k1
  float* X = reinterpret_cast<float*>(&S[0][0][0]);
  static_assert(sizeof(S) >= 4 * 2 * 16 * 64 * 4, "k-group scratch");
  auto xo = [&](int t, int r) { return ((wc * 2 + t) * 16 + r) * 64 + lane; };
  auto round = [&](int src, int dst) __attribute__((always_inline)) {
    if (kg == src) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[xo(t, r)] = acc[t][r];
    }
    __syncthreads();
    if (kg == dst) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += X[xo(t, r)];
    }
    __syncthreads();
  };
  round(3, 1);
  round(2, 0);
  round(1, 0);
  float* outp = slab + (size_t)blockIdx.x * 32 * 256;
  if (kg == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int n = 64 * wc + 8 * (4 * t + (l32 >> 3)) + (l32 & 7);
        outp[co * 256 + n] = acc[t][r];
      }
  }
  if (d_on) bred[dit] = bacc;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
#pragma unroll
    for (int o = 0; o < 10; ++o) t += bred[32 * o + tid];
    slab_bias[(size_t)blockIdx.x * 32 + tid] = t;
  }
}

}  // namespace

// conv1 forward on float observations (SRC_F32) — the rows the fp32 storage plane
// holds (idx gather as ppo_conv1_fwd) — and on raw u8 RGB frames with the
// NormalizeWrapper / FrameStackMono(2) decode fused (SRC_RGB); mbits (nullable):
// the ReLU mask bits of the output as ppo_conv1_fwd_mask writes them
int conv1_fwd_rgb_affine(const uint8_t* frames, const int64_t* idx, long long row0, int B, const float* mean,
                         double stdv, const float* w1, const float* b1, float* out, uint32_t* mbits, void* stream);

int conv1_wgrad_rgb_affine(const float* dz1, const uint8_t* frames, const int64_t* idx, long long row0, int B,
                           const float* mean, double stdv, int Z, float* slab, float* slab_bias, void* stream);

static int conv1_fwd_x6_launch(int src, const void* obs, const int64_t* idx, long long row0, int B, const float* mean,
                               double stdv, const float* w1, const float* b1, float* out, uint32_t* mbits,
                               void* stream) {
  if (B <= 0) return 0;
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || n_cu <= 0)
    n_cu = 256;
  const unsigned nb = (unsigned)(B < n_cu ? B : n_cu);
  const int np = ppo_tune_get("products");
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin(src == SRC_F32 ? "conv1_fwd_f32" : "conv1_fwd_rgb", st, &slot);
  const double rs = 1.0 / stdv;
  const int dbg = ppo_tune_get("stagger") >> 4;   // timing anatomy (kbench --tune stagger=16*dbg)
  // kernel form: fp32 rows take the full-K 10-wave kernel (3.3 vs 3.9 ms per 65,536-image
  // minibatch); RGB frames the K-split 8-wave one (5.8-5.9 vs 6.5 ms: the full-K form's
  // 96 weight VGPRs plus the decode's means spill there)
  const bool ksplit = src == SRC_RGB;
#define L1(S, M, N)                                                                                           \
  if (ksplit) conv1_fwd_x6_kernel<S, M, N><<<nb, 512, 0, st>>>(obs, idx, row0, B, mean, stdv, rs, w1, b1, out, mbits, dbg); \
  else conv1_fwd_x6w_kernel<S, M, N><<<nb, 640, 0, st>>>(obs, idx, row0, B, mean, stdv, rs, w1, b1, out, mbits, dbg)
#define L2(S, N)         \
  if (mbits) { L1(S, true, N); } \
  else { L1(S, false, N); }
#define L3(S)                      \
  if (np == 1) { L2(S, 1); }        \
  else if (np == 9) { L2(S, 9); }   \
  else { L2(S, 6); }
  if (src == SRC_F32) {
    L3(SRC_F32)
  } else {
    L3(SRC_RGB)
  }
#undef L3
#undef L2
#undef L1
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_fwd_x6_kernel");
  return 0;
}

PPO_API int ppo_conv1_fwd_f32(const float* obs, const int64_t* idx, long long row0, int B, const float* w1,
                              const float* b1, float* out, uint32_t* mbits, void* stream) {
  PPO_REQUIRE(B >= 0 && obs != nullptr, "ppo_conv1_fwd_f32: B=%d", B);
  PPO_REQUIRE(((uintptr_t)obs & 15) == 0, "ppo_conv1_fwd_f32: observation rows must be 16-B aligned");
  return conv1_fwd_x6_launch(SRC_F32, obs, idx, row0, B, nullptr, 1.0, w1, b1, out, mbits, stream);
}

PPO_API int ppo_conv1_fwd_rgb(const uint8_t* frames, const int64_t* idx, long long row0, int B, const float* mean,
                              double stdv, const float* w1, const float* b1, float* out, uint32_t* mbits,
                              void* stream) {
  PPO_REQUIRE(B >= 0 && frames != nullptr && stdv != 0.0, "ppo_conv1_fwd_rgb: B=%d std=%g", B, stdv);
  PPO_REQUIRE(((uintptr_t)frames & 15) == 0 && (mean == nullptr || ((uintptr_t)mean & 15) == 0),
              "ppo_conv1_fwd_rgb: frames and mean must be 16-B aligned");
  // the affine fold (rgbaff.hip) unless tuned off or the raw mode's truncated grey plane
  if (ppo_tune_get("rgb_aff") != 0 && !(mean == nullptr && stdv == 1.0))
    return conv1_fwd_rgb_affine(frames, idx, row0, B, mean, stdv, w1, b1, out, mbits, stream);
  return conv1_fwd_x6_launch(SRC_RGB, frames, idx, row0, B, mean, stdv, w1, b1, out, mbits, stream);
}

static int conv1_wgrad_x6_launch(int src, const float* dz1, const void* obs, const int64_t* idx, long long row0, int B,
                                 const float* mean, double stdv, int Z, float* slab, float* slab_bias, void* stream) {
  if (B <= 0 || Z <= 0) return 0;
  PPO_REQUIRE((B + Z - 1) / Z <= WMAXIMG, "conv1 wgrad: %d images over %d blocks (at most %d per block)", B, Z,
              WMAXIMG);
  const int np = ppo_tune_get("products");
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin(src == SRC_F32 ? "conv1_wgrad_f32" : "conv1_wgrad_rgb", st, &slot);
  const double rs = 1.0 / stdv;
  const int dbg = ppo_tune_get("stagger") >> 4;
#define W1(S, N) \
  conv1_wgrad_x6_kernel<S, N><<<Z, 1024, 0, st>>>(dz1, obs, idx, row0, B, mean, stdv, rs, slab, slab_bias, dbg)
#define W2(S)                      \
  if (np == 1) { W1(S, 1); }        \
  else if (np == 9) { W1(S, 9); }   \
  else { W1(S, 6); }
  if (src == SRC_F32) {
    W2(SRC_F32)
  } else {
    W2(SRC_RGB)
  }
#undef W2
#undef W1
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_wgrad_x6_kernel");
  return 0;
}

PPO_API int ppo_conv1_wgrad_f32(const float* dz1, const float* obs, const int64_t* idx, long long row0, int B, int Z,
                                float* slab, float* slab_bias, void* stream) {
  PPO_REQUIRE(B >= 0 && obs != nullptr && ((uintptr_t)obs & 15) == 0,
              "ppo_conv1_wgrad_f32: B=%d, rows must be 16-B aligned", B);
  return conv1_wgrad_x6_launch(SRC_F32, dz1, obs, idx, row0, B, nullptr, 1.0, Z, slab, slab_bias, stream);
}

PPO_API int ppo_conv1_wgrad_rgb(const float* dz1, const uint8_t* frames, const int64_t* idx, long long row0, int B,
                                const float* mean, double stdv, int Z, float* slab, float* slab_bias, void* stream) {
  PPO_REQUIRE(B >= 0 && frames != nullptr && stdv != 0.0, "ppo_conv1_wgrad_rgb: B=%d std=%g", B, stdv);
  PPO_REQUIRE(((uintptr_t)frames & 15) == 0 && (mean == nullptr || ((uintptr_t)mean & 15) == 0),
              "ppo_conv1_wgrad_rgb: frames and mean must be 16-B aligned");
  if (ppo_tune_get("rgb_aff") != 0 && !(mean == nullptr && stdv == 1.0))
    return conv1_wgrad_rgb_affine(dz1, frames, idx, row0, B, mean, stdv, Z, slab, slab_bias, stream);
  return conv1_wgrad_x6_launch(SRC_RGB, dz1, frames, idx, row0, B, mean, stdv, Z, slab, slab_bias, stream);
}

