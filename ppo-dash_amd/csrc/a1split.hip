// conv1 output written pre-split (round 4): the CNNBase trunk's a1 = relu(conv1)
// [B][20][20][32] leaves conv1 as three bf16 planes (a1 = hi + mid + lo exactly,
// the split of DESIGN.md §3) in the 16-B-unit order of conv2's image stage, so
// its two consumers stage it without the per-image split:
//
//   a1s[b] = 4,800 units of 16 B (76,800 B per image): unit (p, c, rho) at
//            (p * 4 + c) * 400 + rho holds channels 8c .. 8c+7 of pixel (y, x)
//            in plane p (0 hi, 1 mid, 2 lo), rho = 100 (2 (y & 1) + (x & 1)) +
//            10 (y >> 1) + (x >> 1) — conv2's parity order (gemm.hip
//            conv2_fwd_x9c_kernel: tap (ky, kx) of output pixel (oy, ox) is
//            pixel rho(oy, ox) + toff(ky, kx)).
//
//   conv1_fwd_split_kernel   conv1_fwd_bf16x3_kernel with the MFMA operands
//                            swapped (weights as A: a lane's four results are
//                            four consecutive channels of one pixel) and the
//                            split in the epilogue: three 8-B stores per tile.
//   conv2_fwd_x9d_kernel     conv2 forward staged by LDS-DMA: the image's 75
//                            1-KB pieces land in the next stage by
//                            global_load_lds_dwordx4 (no VGPRs, no VALU, no
//                            ds_write), issued one image ahead.
//   conv2_wgrad_split_kernel conv2 weight gradient staging the pre-split units
//                            (no split VALU).
//
// Every value is bit-identical to the fp32-a1 path: conv1's sums are the same
// MFMA products (swapped operands), the split is split8's arithmetic, and the
// consumers' products and summation orders are unchanged.
// Reference: CNNBase conv1 -> conv2, T/a2c_ppo_acktr/model.py:177-180.
#include "igemm_x9.h"

int gemm_products();     // gemm.hip: ppo_tune_set("products") value
int gemm_device_cus();   // gemm.hip: persistent-grid size

namespace {

constexpr int A1S_UNITS = 4800, A1S_BYTES = 16 * A1S_UNITS;

__device__ __forceinline__ int c2_rho(int y, int x) {
  return 100 * (2 * (y & 1) + (x & 1)) + 10 * (y >> 1) + (x >> 1);
}

// split8's arithmetic on four values -> three 8-B groups of bf16 (hi, mid, lo)
__device__ __forceinline__ void split4(const float v[4], uint2& h, uint2& m, uint2& l) {
  float r[4];
  uint32_t hw[2], mw[2], lw[2];
#pragma unroll
  for (int j = 0; j < 4; j += 2) {
    const bf16x2 hh = __builtin_convertvector(f32x2{v[j], v[j + 1]}, bf16x2);
    hw[j >> 1] = __builtin_bit_cast(uint32_t, hh);
    r[j] = v[j] - (float)hh[0];
    r[j + 1] = v[j + 1] - (float)hh[1];
    const bf16x2 mm = __builtin_convertvector(f32x2{r[j], r[j + 1]}, bf16x2);
    mw[j >> 1] = __builtin_bit_cast(uint32_t, mm);
    const float r0 = r[j] - (float)mm[0], r1 = r[j + 1] - (float)mm[1];
    const bf16x2 ll = __builtin_convertvector(f32x2{r0, r1}, bf16x2);
    lw[j >> 1] = __builtin_bit_cast(uint32_t, ll);
  }
  h = uint2{hw[0], hw[1]};
  m = uint2{mw[0], mw[1]};
  l = uint2{lw[0], lw[1]};
}

// One 1-KB LDS-DMA piece: lane l's 16 B from gsrc land at LDS byte lds_dst + 16 l.
// Inline asm, so the compiler's waitcnt pass does not see it and inserts no
// vmcnt(0) before the LDS reads of the other stage (the collapse DESIGN.md §6
// records for the builtin); every wave retires its own pieces with an explicit
// vmcnt before the barrier that publishes them.  M0 is saved and restored in
// the same statement (it is compiler-reserved).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>(p);
}

// ---------------------------------------------------------------------------
// conv1 forward (u8 observations, C = 4) writing a1s: conv1_fwd_bf16x3_kernel's
// structure (one persistent block per CU walking images, image in LDS as bf16,
// weights split once per block into registers), MFMA operands swapped so that
// lane (i16, g) of row tile rt holds channels 16 ct + 4g .. +3 of pixel
// 16 rt + i16.  MASK: the ReLU mask bits of the conv2 dgrad (u16 [B][400][2],
// bit j of word (p, ct) = channel 16 ct + j of pixel p > 0), as the fp32 path.
// ---------------------------------------------------------------------------
template <bool MASK>
__global__ __launch_bounds__(512) void conv1_fwd_split_kernel(const uint8_t* __restrict__ obs,
                                                              const int64_t* __restrict__ idx, long long row0,
                                                              int B, const float* __restrict__ w,
                                                              const float* __restrict__ bias,
                                                              uint16_t* __restrict__ a1s,
                                                              uint16_t* __restrict__ mbits) {
  constexpr int C = 4, IMG = 84, IMG2 = IMG * IMG;
  constexpr int NPX = C * IMG2, CH = NPX / 16, K = C * 64, KS = K / 32, PER = (CH + 511) / 512, NT = 7;
  __shared__ __attribute__((aligned(16))) uint16_t img[2][NPX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, rq = wave >> 1, ntile = rq == 0 ? 7 : 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int col = ct * 16 + i16;
  const f32x4 bv4 = *reinterpret_cast<const f32x4*>(bias + ct * 16 + 4 * g);
  bf16x8 wf[3][KS];   // this lane's weight row (channel col), split once per block
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const float* wp = w + (size_t)col * K + 32 * s + 8 * g;
    uint32_t h[8], m[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) split_bf16x3(wp[j], h[j], m[j], l[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wf[0][s][j] = __builtin_bit_cast(__bf16, (uint16_t)h[j]);
      wf[1][s][j] = __builtin_bit_cast(__bf16, (uint16_t)m[j]);
      wf[2][s][j] = __builtin_bit_cast(__bf16, (uint16_t)l[j]);
    }
  }
  // output units of this lane per row tile: pixel 16 rt + i16, channel chunk 2 ct + (g >> 1), half g & 1
  int uoff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int px = (rq + 4 * t) * 16 + i16, oy = px / 20, ox = px - 20 * oy;
    uoff[t] = ((2 * ct + (g >> 1)) * 400 + c2_rho(oy, ox)) * 16 + (g & 1) * 8;
  }
  uint4 stage[PER];
  auto fetch = [&](int b) {
    const uint4* src = reinterpret_cast<const uint4*>(obs + obs_row(idx, row0, b) * (long long)NPX);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = tid + 512 * j;
      if (c < CH) stage[j] = src[c];
    }
  };
  auto put = [&](int buf) {   // u8 -> bf16 (exact)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = tid + 512 * j;
      if (c < CH) {
        const uint32_t v[4] = {stage[j].x, stage[j].y, stage[j].z, stage[j].w};
        uint32_t o[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 f = to_f32x4(v[q]);
          o[2 * q] = __builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u);
          o[2 * q + 1] = __builtin_amdgcn_perm(__float_as_uint(f[3]), __float_as_uint(f[2]), 0x07060302u);
        }
        uint4* d = reinterpret_cast<uint4*>(img[buf] + 16 * c);
        d[0] = uint4{o[0], o[1], o[2], o[3]};
        d[1] = uint4{o[4], o[5], o[6], o[7]};
      }
    }
  };
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
    put(0);
    if (b + G < B) fetch(b + G);
  }
  __syncthreads();
  for (; b < B; b += G) {
    if (b + G < B) put(cur ^ 1);
    if (b + 2 * G < B) fetch(b + 2 * G);
    const uint16_t* I = img[cur];
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = zero4();
    int pix[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int row = (rq + 4 * t) * 16 + i16, oy = row / 20, ox = row - oy * 20;
      pix[t] = oy * (4 * IMG) + ox * 4;
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k0 = 32 * s + 8 * g;
      const uint16_t* Is = I + (k0 >> 6) * IMG2 + ((k0 >> 3) & 7) * IMG;
      bf16x8 a[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t < ntile) {
          const uint2* p2 = reinterpret_cast<const uint2*>(Is + pix[t]);
          const uint2 lo = p2[0], hi = p2[1];
          a[t] = __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y});
        }
#pragma unroll
      for (int part = 0; part < 3; ++part)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (t < ntile) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[part][s], a[t], acc[t], 0, 0, 0);
    }
    char* ob = reinterpret_cast<char*>(a1s) + (size_t)b * A1S_BYTES;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (t < ntile) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(acc[t][r] * (1.0f / 255.0f) + bv4[r], 0.f);
        uint2 h, m, l;
        split4(v, h, m, l);
        *reinterpret_cast<uint2*>(ob + uoff[t]) = h;
        *reinterpret_cast<uint2*>(ob + uoff[t] + 1600 * 16) = m;
        *reinterpret_cast<uint2*>(ob + uoff[t] + 3200 * 16) = l;
        if constexpr (MASK) {   // bits 4g .. 4g+3 of pixel 16 rt + i16's word ct, combined over g
          int nib = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) nib |= (v[r] > 0.f ? 1 : 0) << r;
          const int w16 = nib | (__shfl_down(nib, 16, 64) << 4) | (__shfl_down(nib, 32, 64) << 8) |
                          (__shfl_down(nib, 48, 64) << 12);
          if (g == 0) mbits[((size_t)b * 400 + (rq + 4 * t) * 16 + i16) * 2 + ct] = (uint16_t)w16;
        }
      }
    __syncthreads();
    cur ^= 1;
  }
}

// ---------------------------------------------------------------------------
// conv2 forward from a1s, staged by LDS-DMA.  Compute, wave roles, LDS layout
// and epilogue are conv2_fwd_x9c_kernel's (gemm.hip): wave w = n tile w & 3 x
// K half w >> 2 (taps 8 kh .. +7, weights pre-split in registers), six row
// tiles of 16 output pixels, K halves summed through the lo plane of the stage
// the image has just left.  Staging: two stages of 76,800 B; image b + 2G's
// 75 pieces are issued at the end of image b into b's stage:
//   * after barrier B, the K-half-1 waves (which have just written their
//     partials) issue the hi / mid planes (pieces 0-49, 13 per wave, clamped);
//   * each K-half-0 wave nt reads its partials (6 KB = lo-plane pieces 6 nt ..
//     6 nt + 5), retires the reads (lgkmcnt(0)) and then issues exactly those
//     pieces (wave 3 also piece 24 of the plane, beyond the partials);
//   * every wave retires its pieces (vmcnt(0): they were issued a whole image
//     earlier) before barrier A of image b + G, which publishes them.
// So the DMA has one image's compute to land, no register or VALU is spent on
// staging, and each image needs two barriers.
// ---------------------------------------------------------------------------
template <int NP, bool MASK>
__global__ __launch_bounds__(512) void conv2_fwd_x9d_kernel(const uint16_t* __restrict__ a1s, int B,
                                                           const uint16_t* __restrict__ wpl,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ out,
                                                           uint16_t* __restrict__ mbits) {
  constexpr int U = 400, PLN = 4 * U, STG = 3 * PLN, MT = 6, KS = 8, WN = 64 * 512;
  constexpr int STG_B = STG * 16;
  __shared__ __attribute__((aligned(16))) bf16x8 S[2 * STG];
  __shared__ int vtab[MT][16];
  __shared__ int otab[MT][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int nt = wave & 3, kh = wave >> 2, co = 16 * nt + i16;
  if (tid < 16) {
    int t = 0;
    for (int v = tid; v <= 88; v += 16)
      if (v % 10 != 9) {
        vtab[t][tid] = v;
        otab[t][tid] = 9 * (v / 10) + v % 10;
        ++t;
      }
    for (; t < MT; ++t) {
      vtab[t][tid] = tid;
      otab[t][tid] = -1;
    }
  }
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + co * 512 + (8 * kh + s) * 32 + 8 * g);
  const f32x4 bv4 = *reinterpret_cast<const f32x4*>(bias + 16 * nt + 4 * g);
  wait_vm0();
  const uint32_t sbase = lds_addr(S);
  auto piece = [&](int b, int st, int k) {   // 1-KB piece k (0..74) of image b into stage st
    const char* src = reinterpret_cast<const char*>(a1s) + (size_t)b * A1S_BYTES + k * 1024 + lane * 16;
    glds16(src, __builtin_amdgcn_readfirstlane(sbase + st * STG_B + k * 1024));
  };
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {   // images b and b + G: pieces wave + 8 i (clamped: harmless duplicates)
    if (b < B) piece(b, 0, min(wave + 8 * i, 74));
    if (b + G < B) piece(b + G, 1, min(wave + 8 * i, 74));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // stages 0 / 1 and vtab / otab
  int vrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) vrow[t] = vtab[t][i16] + g * U;
  for (; b < B; b += G) {
    const bf16x8* Sc = S + cur * STG;
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = zero4();
    // software-pipelined over half k-steps (group gi = k-step gi >> 1, row tiles
    // 3 (gi & 1) .. +2): group gi + 1's nine fragment reads are issued before group
    // gi's MFMAs (the registers freed by the DMA staging hold them)
    Frag3 A[2][3];
    auto load_grp = [&](int gi, Frag3 (&a)[3]) {
      const int tap = 8 * kh + (gi >> 1), ky = tap >> 2, kx = tap & 3, t0 = 3 * (gi & 1);
      const int toff = 100 * (2 * (ky & 1) + (kx & 1)) + 10 * (ky >> 1) + (kx >> 1);
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const bf16x8* q = Sc + vrow[t0 + u] + toff;
        a[u].h = q[0];
        a[u].m = q[PLN];
        a[u].l = q[2 * PLN];
      }
    };
    load_grp(0, A[0]);
#pragma unroll
    for (int gi = 0; gi < 2 * KS; ++gi) {
      if (gi + 1 < 2 * KS) load_grp(gi + 1, A[(gi + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of this group's MFMAs
      const int s = gi >> 1, t0 = 3 * (gi & 1);
      const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
      const Frag3(&a)[3] = A[gi & 1];
#define PPO_PART(X, Y) \
  _Pragma("unroll") for (int u = 0; u < 3; ++u) acc[t0 + u] = mma(w.Y, a[u].X, acc[t0 + u]);
      PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
      __builtin_amdgcn_sched_barrier(0);
    }
    // this wave's pieces of image b + G (issued one image ago) and its stores have retired
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();   // A: stage cur consumed; stage cur ^ 1 published
    f32x4* R = reinterpret_cast<f32x4*>(S + cur * STG + 2 * PLN);   // partials in the lo plane just left
    if (kh == 1) {
#pragma unroll
      for (int t = 0; t < MT; ++t) R[(nt * MT + t) * 64 + lane] = acc[t];
    }
    lds_barrier();   // B: partials in LDS
    const int b2 = b + 2 * G;
    if (kh == 1) {
      if (b2 < B) {
#pragma unroll
        for (int i = 0; i < 13; ++i) piece(b2, cur, min(nt + 4 * i, 49));   // hi / mid planes
      }
    } else {
      f32x4 pr[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) pr[t] = R[(nt * MT + t) * 64 + lane];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's partial region is read
      if (b2 < B) {
#pragma unroll
        for (int i = 0; i < 6; ++i) piece(b2, cur, 50 + 6 * nt + i);
        if (nt == 3) piece(b2, cur, 74);
      }
      const auto rs = make_rsrc(out + (size_t)b * (81 * 64), 81 * 64 * 4);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const f32x4 v = acc[t] + pr[t];
        const int m = otab[t][i16];
        f32x4 y;
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + bv4[r], 0.f);
        bstore_f32x4(y, rs, m >= 0 ? 4 * (m * 64 + 16 * nt + 4 * g) : -1);
        if constexpr (MASK) {
          int nib = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) nib |= (y[r] > 0.f ? 1 : 0) << r;
          const int w16 = nib | (__shfl_down(nib, 16, 64) << 4) | (__shfl_down(nib, 32, 64) << 8) |
                          (__shfl_down(nib, 48, 64) << 12);
          if (g == 0 && m >= 0) mbits[((size_t)b * 81 + m) * 4 + nt] = (uint16_t)w16;
        }
      }
    }
    cur ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// conv2 weight gradient from a1s: conv2_wgrad_x9_kernel (gemm.hip) with the X
// staging reading the pre-split units (three 16-B loads per unit instead of
// two fp32 loads and the split).  X [3][400 px Q][32 ci], Q = 20 y + 10 (x & 1)
// + (x >> 1), 8-B unit u of pixel Q at u ^ 4 ((Q >> 3) & 1); D = dz2 split and
// transposed; one stage, the next image in registers.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int c2w_pix_s(int r) {
  r = r < 80 ? r : 80;
  return r < 72 ? (r >> 3) * 9 + (r & 7) : (r - 72) * 9 + 8;
}

template <int NP>
__global__ __launch_bounds__(512) void conv2_wgrad_split_kernel(const float* __restrict__ dz2,
                                                               const uint16_t* __restrict__ a1s, int B,
                                                               float* __restrict__ slab,
                                                               float* __restrict__ slab_bias) {
  constexpr int XPL = 400 * 32, DR = 112, DPL = 64 * DR;
  constexpr int XU = 1600, XPER = (XU + 511) / 512, DU = 64 * 12, DPER = (DU + 511) / 512;
  __shared__ __attribute__((aligned(16))) uint16_t X[3 * XPL];
  __shared__ __attribute__((aligned(16))) uint16_t D[3 * DPL];
  __shared__ float bred[512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int q = i16 >> 2, p = i16 & 3;
  int Qb[3][2];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = c2w_pix_s(32 * s + 8 * g + 4 * h + q), oy = m / 9;
      Qb[s][h] = 40 * oy + (m - 9 * oy);
    }
  // X unit u = tid + 512 j -> pixel Q = u >> 2, chunk c = u & 3; its three planes come
  // from a1s units (pl, c, rho(Q)) = pl * 1600 + c * 400 + rho
  int xsrc[XPER], xdst[XPER];
#pragma unroll
  for (int j = 0; j < XPER; ++j) {
    const int u = min(tid + 512 * j, XU - 1), Q = u >> 2, c = u & 3, y = Q / 20, rem = Q - 20 * y;
    const int x = rem < 10 ? 2 * rem : 2 * (rem - 10) + 1;
    xsrc[j] = c * 400 + c2_rho(y, x);
    xdst[j] = Q * 32 + 8 * (c ^ (((Q >> 3) & 1) * 2));
  }
  u32x4_t xs[XPER][3];
  float ds[DPER][8];
  float bsum = 0.f;
  auto fetch = [&](int b) {
    const u32x4_t* src = reinterpret_cast<const u32x4_t*>(a1s) + (size_t)b * A1S_UNITS;
#pragma unroll
    for (int j = 0; j < XPER; ++j)
      if (tid + 512 * j < XU) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) xs[j][pl] = src[pl * 1600 + xsrc[j]];
      }
    const float* dsrc = dz2 + (size_t)b * (81 * 64);
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int v = tid + 512 * j;
      if (v < DU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int r = 8 * (v >> 6) + e;
          ds[j][e] = r < 81 ? dsrc[c2w_pix_s(r) * 64 + (v & 63)] : 0.f;
        }
      }
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int j = 0; j < XPER; ++j)
      if (tid + 512 * j < XU) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x4_t*>(&X[pl * XPL + xdst[j]]) = xs[j][pl];
      }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int v = tid + 512 * j;
      if (v < DU) {
        Frag3 f;
        split8(f32x4{ds[j][0], ds[j][1], ds[j][2], ds[j][3]}, f32x4{ds[j][4], ds[j][5], ds[j][6], ds[j][7]}, f,
               false);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += ds[j][e];
        const int off = (v & 63) * DR + 8 * (v >> 6);
        *reinterpret_cast<bf16x8*>(&D[off]) = f.h;
        *reinterpret_cast<bf16x8*>(&D[DPL + off]) = f.m;
        *reinterpret_cast<bf16x8*>(&D[2 * DPL + off]) = f.l;
      }
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[j][mt] = zero4();
  const int Z = gridDim.x;
  int b = blockIdx.x;
  if (b < B) {
    fetch(b);
    put();
    if (b + Z < B) fetch(b + Z);
  }
  __syncthreads();
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  for (; b < B; b += Z) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      Frag3 a[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int off = (16 * mt + i16) * DR + 32 * s + 8 * g;
        a[mt].h = *reinterpret_cast<const bf16x8*>(&D[off]);
        a[mt].m = *reinterpret_cast<const bf16x8*>(&D[DPL + off]);
        a[mt].l = *reinterpret_cast<const bf16x8*>(&D[2 * DPL + off]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int tap = 2 * wave + (j >> 1), ky = tap >> 2, kx = tap & 3, cb = j & 1;
        const int toff = 20 * ky + 10 * (kx & 1) + (kx >> 1);
        s16x4 t[3][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int Q = Qb[s][h] + toff, unit = (4 * cb + p) ^ (((Q >> 3) & 1) * 4);
          const uint16_t* rp = &X[Q * 32 + 4 * unit];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            t[pl][h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(rp + pl * XPL));
        }
        Frag3 bf;
        bf.h = __builtin_bit_cast(bf16x8, __builtin_shufflevector(t[0][0], t[0][1], 0, 1, 2, 3, 4, 5, 6, 7));
        bf.m = __builtin_bit_cast(bf16x8, __builtin_shufflevector(t[1][0], t[1][1], 0, 1, 2, 3, 4, 5, 6, 7));
        bf.l = __builtin_bit_cast(bf16x8, __builtin_shufflevector(t[2][0], t[2][1], 0, 1, 2, 3, 4, 5, 6, 7));
#define PPO_PART(XX, YY) \
  _Pragma("unroll") for (int mt = 0; mt < 4; ++mt) acc[j][mt] = mma(a[mt].XX, bf.YY, acc[j][mt]);
        PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
      }
    }
    __syncthreads();
    if (b + Z < B) put();
    if (b + 2 * Z < B) fetch(b + 2 * Z);
    __syncthreads();
  }
  float* o = slab + (size_t)blockIdx.x * (64 * 512) + 64 * wave + i16;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(16 * mt + 4 * g + r) * 512 + 16 * j] = acc[j][mt][r];
  bred[tid] = bsum;
  __syncthreads();
  if (tid < 64) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) t += bred[tid + 64 * w];
    slab_bias[(size_t)blockIdx.x * 64 + tid] = t;
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI (include/ppo_hip.h)
// ---------------------------------------------------------------------------
PPO_API long long ppo_a1s_bytes(int B) { return (long long)B * A1S_BYTES; }

PPO_API int ppo_conv1_fwd_split(const uint8_t* obs, const int64_t* idx, long long row0, int B, const float* w1,
                                const float* b1, uint16_t* a1s, uint32_t* mbits, void* stream) {
  PPO_REQUIRE(B >= 0 && obs && w1 && b1 && a1s, "ppo_conv1_fwd_split: B=%d", B);
  PPO_REQUIRE(gemm_products() != 1, "ppo_conv1_fwd_split: the split a1 path needs fp32 arithmetic (products 6 / 9)");
  PPO_REQUIRE(((uintptr_t)a1s & 15) == 0, "ppo_conv1_fwd_split: a1s must be 16-B aligned");
  if (B == 0) return 0;
  const int n_cu = gemm_device_cus();
  const unsigned nb = (unsigned)(B < n_cu ? B : n_cu);
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin("conv1_fwd_u8", st, &slot);
  if (mbits)
    conv1_fwd_split_kernel<true><<<nb, 512, 0, st>>>(obs, idx, row0, B, w1, b1, a1s,
                                                     reinterpret_cast<uint16_t*>(mbits));
  else
    conv1_fwd_split_kernel<false><<<nb, 512, 0, st>>>(obs, idx, row0, B, w1, b1, a1s, nullptr);
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_fwd_split_kernel");
  return 0;
}

PPO_API int ppo_conv2_fwd_split(const uint16_t* a1s, int B, const float* w2p, const float* b2, float* out,
                                uint64_t* mbits, void* stream) {
  PPO_REQUIRE(B >= 0 && a1s && w2p && b2 && out, "ppo_conv2_fwd_split: B=%d", B);
  const int np = gemm_products();
  PPO_REQUIRE(np != 1, "ppo_conv2_fwd_split: the split a1 path needs fp32 arithmetic (products 6 / 9)");
  PPO_REQUIRE(((uintptr_t)a1s & 15) == 0, "ppo_conv2_fwd_split: a1s must be 16-B aligned");
  if (B == 0) return 0;
  const int n_cu = gemm_device_cus();
  const unsigned nb = (unsigned)(B < n_cu ? B : n_cu);
  hipStream_t st = as_stream(stream);
  const uint16_t* wpl = reinterpret_cast<const uint16_t*>(w2p + 64 * 512);   // the packed segment's planes
  uint16_t* mb = reinterpret_cast<uint16_t*>(mbits);
  int slot;
  const bool prof = ppo_prof_begin("conv2_fwd", st, &slot);
  if (np == 9) {
    if (mb) conv2_fwd_x9d_kernel<9, true><<<nb, 512, 0, st>>>(a1s, B, wpl, b2, out, mb);
    else conv2_fwd_x9d_kernel<9, false><<<nb, 512, 0, st>>>(a1s, B, wpl, b2, out, nullptr);
  } else {
    if (mb) conv2_fwd_x9d_kernel<6, true><<<nb, 512, 0, st>>>(a1s, B, wpl, b2, out, mb);
    else conv2_fwd_x9d_kernel<6, false><<<nb, 512, 0, st>>>(a1s, B, wpl, b2, out, nullptr);
  }
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 81 * 64 * 512);
  PPO_LAUNCH_CHECK("conv2_fwd_x9d_kernel");
  return 0;
}

PPO_API int ppo_conv2_wgrad_split(const float* dz2, const uint16_t* a1s, int B, int Z, float* slab,
                                  float* slab_bias, void* stream) {
  PPO_REQUIRE(B > 0 && Z > 0 && dz2 && a1s && slab && slab_bias, "ppo_conv2_wgrad_split: B=%d Z=%d", B, Z);
  const int np = gemm_products();
  PPO_REQUIRE(np != 1, "ppo_conv2_wgrad_split: the split a1 path needs fp32 arithmetic (products 6 / 9)");
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin("conv2_wgrad", st, &slot);
  if (np == 9) conv2_wgrad_split_kernel<9><<<Z, 512, 0, st>>>(dz2, a1s, B, slab, slab_bias);
  else conv2_wgrad_split_kernel<6><<<Z, 512, 0, st>>>(dz2, a1s, B, slab, slab_bias);
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 81 * 64 * 512);
  PPO_LAUNCH_CHECK("conv2_wgrad_split_kernel");
  return 0;
}
