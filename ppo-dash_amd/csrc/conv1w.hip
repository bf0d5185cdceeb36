// conv1 weight gradient on u8 observations, k-split over waves (round 4;
// ppo_tune_set("conv1_wgrad", 8); the default since round 5 is its one-wave-per-SIMD
// form below, tune 9):
//   dW1[co][(c, ky, kx)] = Σ_images Σ_px dz1[px][co] · u[c][4oy+ky][4ox+kx]
// (the conv1 backward of CNNBase, T/a2c_ppo_acktr/model.py:177), exact: u8 pixels
// are exact in bf16 and dz = hi + mid + lo (split_bf16x3), three
// v_mfma_f32_32x32x16_bf16 products per block pair with fp32 accumulation
// (DESIGN.md §3).  Replaces the part-pipelined kernel's structure:
//
//   * one persistent block (8 waves) per CU walks images; every wave owns ALL
//     eight 32-column tiles of the 32 x 256 gradient (128 accumulator VGPRs) and
//     an eighth of the image's 25 k-steps of 16 pixels (k-steps w,
//     w + 8, w + 16, and tile w of k-step 24): the per-image work of every wave
//     is the same 75 MFMAs, and the eight partial gradients are summed once per
//     block at the end (fixed order), not per image;
//   * dz never passes through LDS: each wave loads its k-step's A fragment (8
//     consecutive pixels of one channel per lane: pixels 16 s + 8 h .. +7 are
//     contiguous in the [px][co] layout) straight from HBM one k-step ahead and
//     splits it in registers — no staging writes, no split by other waves;
//   * the image is converted from u8 to bf16 ONCE per image (not once per kx)
//     into "phase rows": E[c][y][dx][X] = u[c][y][4X + dx], so tap (ky, kx) of
//     output pixel (oy, ox) is E[c][4oy+ky][kx & 3][ox + (kx >> 2)]: a lane's
//     four pixels of an output-row quad are four consecutive elements; the
//     kx >= 4 half reads them one element later, realigned with two
//     v_alignbyte (8-B read + 4-B read per quad);
//   * two E stages (2 x 64,512 B); the next image's raw u8 bytes arrive by
//     LDS-DMA into a 28-KB buffer beside them and are converted into the other
//     stage mid-image (schedule below).  A first form held the next image in
//     registers (tune 7, 1.674-1.680 ms per c3 minibatch against 1.597; removed
//     in round 5, see DESIGN.md §6 run records).
// Output: the split-K slab [Z][32][256] of u8-integer sums (the reduce applies
// 1/255) and bias partials [Z][32], as every conv1 wgrad variant.
#include "igemm_x9.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));


// The same algorithm with the u8 image staged by LDS-DMA (ppo_tune_set("conv1_wgrad", 8)):
// the raw image (28,224 B) lands in a 28-KB LDS buffer beside the two E stages
// (157,696 B in all), so no VGPRs hold the next image and the freed registers
// carry the dz fragments two k-steps ahead (four 8-value buffers).  Per image b:
//   k-steps A (s = w), B (s = w + 8);  barrier Y: raw(b + G) visible (its DMA
//   retired: in issue order it is older than the dz loads k-step B waited for);
//   convert raw -> E[other stage];  barrier Z: raw consumed, E[other] complete;
//   dz loads of image b + G's k-steps A, B;  DMA of raw(b + 2G) (after those
//   loads, so no compiler wait before k-step D drains it);  k-steps C (s = w +
//   16), D (k-step 24, tile w).  Two barriers per image.
template <int NW>
__global__ __launch_bounds__(NW * 64) void conv1_wgrad_kw2_kernel(const float* __restrict__ dz1,
                                                                 const uint8_t* __restrict__ obs,
                                                                 const int64_t* __restrict__ idx, long long row0,
                                                                 int B, float* __restrict__ slab,
                                                                 float* __restrict__ slab_bias) {
  static_assert(NW == 8, "8 waves");
  constexpr int C = 4, IMG = 84, IMGB = C * IMG * IMG;
  constexpr int XW = 24, ROWE = 4 * XW, EST = C * IMG * ROWE;
  constexpr int NITEM = C * IMG * 6, IPER = (NITEM + NW * 64 - 1) / (NW * 64);
  constexpr int RAWB = 28 * 1024;                          // raw u8 image buffer (28 pieces)
  __shared__ __attribute__((aligned(16))) uint16_t E[2 * EST + RAWB / 2];   // 157,696 B
  uint8_t* const RAW = reinterpret_cast<uint8_t*>(E + 2 * EST);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int G = gridDim.x;
  const int kx = l32 & 7, dxl = kx & 3, sh = 2 * (kx >> 2);
  const int lbase = ((l32 >> 3) * 4 + dxl) * XW;
  const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(RAW);
  auto dma_raw = [&](int b) {   // pieces wave + 8 i (i < 4), clamped: harmless duplicates / tail
    const uint8_t* img = obs + obs_row(idx, row0, b) * (long long)IMGB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = min(wave + 8 * i, 27);
      const int off = min(pc * 1024 + lane * 16, IMGB - 16);
      glds16(img + off, __builtin_amdgcn_readfirstlane(raw_lds + pc * 1024));
    }
  };
  auto put = [&](int st) {   // RAW -> E[st]: u8 -> bf16 (exact), de-interleaved by x mod 4
    uint16_t* S = E + st * EST;
#pragma unroll
    for (int j = 0; j < IPER; ++j) {
      const int it = tid + NW * 64 * j;
      if (it >= NITEM) break;
      const int r = it / 6, g6 = it - 6 * r, src = r * IMG + 16 * g6;
      const uint32_t* rp = reinterpret_cast<const uint32_t*>(RAW + src);
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = src + 4 * k < IMGB ? rp[k] : 0u;
      uint16_t* dp = S + r * ROWE + 4 * g6;
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        float f[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) f[k] = (float)((w[k] >> (8 * dx)) & 255u);
        const uint2 q = {__builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u),
                         __builtin_amdgcn_perm(__float_as_uint(f[3]), __float_as_uint(f[2]), 0x07060302u)};
        *reinterpret_cast<uint2*>(dp + dx * XW) = q;
      }
    }
  };
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bacc = 0.f;
  // one dz_load = DZ_LOADS single-dword buffer loads (128 B apart, so never merged);
  // the vmcnt of barrier Y below counts them
  constexpr int DZ_LOADS = 8;
  auto dz_load = [&](int b, int s, float (&d)[DZ_LOADS]) {
    const auto rs = make_rsrc(dz1 + (size_t)b * 12800, 12800 * 4);
    const int o = ((16 * s + 8 * h) * 32 + l32) * 4;
#pragma unroll
    for (int j = 0; j < DZ_LOADS; ++j) d[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o + 128 * j, 0, 0));
  };
  auto bfrag = [&](const uint16_t* S, int tt, int q0off, int q1off) {
    const int toff = ((tt >> 1) * IMG + 4 * (tt & 1)) * ROWE + lbase;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint16_t* p = S + toff + (k ? q1off : q0off);
      const uint2 d01 = *reinterpret_cast<const uint2*>(p);
      const uint32_t d2 = *reinterpret_cast<const uint32_t*>(p + 4);
      o[2 * k] = __builtin_amdgcn_alignbyte(d01.y, d01.x, sh);
      o[2 * k + 1] = __builtin_amdgcn_alignbyte(d2, d01.y, sh);
    }
    return __builtin_bit_cast(bf16x8, uint4{o[0], o[1], o[2], o[3]});
  };
  auto qoff = [&](int q) { const int oy = q / 5; return 4 * oy * ROWE + 4 * (q - 5 * oy); };
  auto kstep = [&](const uint16_t* S, int s, const float (&d)[8], int t0, int t1) {
    Frag3 a;
    split8(f32x4{d[0], d[1], d[2], d[3]}, f32x4{d[4], d[5], d[6], d[7]}, a, false);
    const int q0 = 4 * s + 2 * h, o0 = qoff(q0), o1 = qoff(q0 + 1);
#pragma unroll
    for (int tt = 0; tt < 8; ++tt) {
      if (tt < t0 || tt >= t1) continue;
      const bf16x8 bq = bfrag(S, tt, o0, o1);
      acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, bq, acc[tt], 0, 0, 0);
      acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, bq, acc[tt], 0, 0, 0);
      acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, bq, acc[tt], 0, 0, 0);
    }
  };
  auto add8 = [&](const float (&d)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) bacc += d[j];
  };
  int b = blockIdx.x, cur = 0;
  float dA[DZ_LOADS], dB[DZ_LOADS], dC[DZ_LOADS], dD[DZ_LOADS];
  if (b < B) {
    dma_raw(b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    put(0);
    __syncthreads();   // raw consumed, E[0] complete
    dz_load(b, wave, dA);
    dz_load(b, wave + 8, dB);
    if (b + G < B) dma_raw(b + G);
  }
  for (; b < B; b += G) {
    const uint16_t* S = E + cur * EST;
    const bool nxt = b + G < B;
    dz_load(b, wave + 16, dC);
    kstep(S, wave, dA, 0, 8);
    add8(dA);
    dz_load(b, 24, dD);
    kstep(S, wave + 8, dB, 0, 8);
    add8(dB);
    if (nxt) {
      // raw(b + G)'s DMA was issued after dA / dB's loads of image b + G (previous
      // iteration, or the prologue) and before this iteration's dz_load(dC) and
      // dz_load(dD); both asm statements clobber memory, so the compiler moves no
      // load across them and exactly those 2 * DZ_LOADS loads are younger than the
      // DMA: vmcnt(2 * DZ_LOADS) retires the DMA and leaves dC, dD in flight
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DZ_LOADS) : "memory");
      lds_barrier();   // Y: every wave's pieces of raw(b + G) are in LDS
      put(cur ^ 1);
      lds_barrier();   // Z: raw consumed, E[cur ^ 1] complete
      dz_load(b + G, wave, dA);
      dz_load(b + G, wave + 8, dB);
      if (b + 2 * G < B) dma_raw(b + 2 * G);
    }
    kstep(S, wave + 16, dC, 0, 8);
    add8(dC);
    kstep(S, 24, dD, wave, wave + 1);
    if (wave == 0) add8(dD);
    cur ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* X = reinterpret_cast<float*>(E);
#pragma unroll
  for (int half = 4; half >= 1; half >>= 1)
#pragma unroll
    for (int t0 = 0; t0 < 8; t0 += 4) {
      if (wave >= half && wave < 2 * half) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) X[(((wave - half) * 4 + t) * 16 + r) * 64 + lane] = acc[t0 + t][r];
      }
      __syncthreads();
      if (wave < half) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t0 + t][r] += X[((wave * 4 + t) * 16 + r) * 64 + lane];
      }
      __syncthreads();
    }
  float* out = slab + (size_t)blockIdx.x * 32 * 256;
  if (wave == 0) {
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = (r & 3) + 8 * (r >> 2) + 4 * h, n = 32 * t + l32;
        out[co * 256 + n] = acc[t][r];
      }
  }
  X[tid] = bacc;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += X[w * 64 + tid] + X[w * 64 + 32 + tid];
    slab_bias[(size_t)blockIdx.x * 32 + tid] = t;
  }
}

// The same product with ONE wave per SIMD (round 5, ppo_tune_set("conv1_wgrad", 9),
// the default).  kw2's anatomy shows a chain of latencies per wave —
// one tile of B read-ahead, the dz split in front of each k-step, a conversion phase
// between two barriers — that its 256-VGPR budget leaves no room to pipeline.  Here
// 4 waves with 512 registers each (accumulators in AGPRs):
//   * wave w: k-steps w + 4 i (i < 6) of every image and tiles 2 w, 2 w + 1 of
//     k-step 24: 150 MFMAs per wave per image;
//   * B fragments read RA tiles ahead through a ring (one flat sequence of the 50
//     tiles of the image); the dz split of step i + 1 (and of the next image's step
//     0) computed during step i; the dz slots and the next image's u8 bytes
//     prefetched into registers a few steps ahead (schedule at the loop);
//   * the next image converted into the other E stage during this image's steps,
//     one or two 16-B items per step (plain buffer loads: no raw LDS buffer, no
//     DMA): one barrier per image.
// The slab format and the sums are kw2's (a different summation order: not
// bit-identical to tune 8).  kbench at Z = 256: 1.48-1.50 vs 1.585-1.59 ms.
#ifndef KW3_BXT
#define KW3_BXT 1
#endif
#ifndef KW3_FENCE
#define KW3_FENCE 1
#endif
#ifndef KW3_RA
#define KW3_RA 3   // B read-ahead in tiles (lgkmcnt holds 15: 4 reads per tile)
#endif
// NW = 4: one wave per SIMD, all 8 column tiles per wave (tune 9); NW = 8: two waves
// per SIMD, wave w = 2 kg + ch owning column tiles 4 ch .. 4 ch + 3 of the k-steps of
// group kg (the pair kg splits the same dz; tune 10)
template <int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4))) void conv1_wgrad_kw3_kernel(
    const float* __restrict__ dz1, const uint8_t* __restrict__ obs, const int64_t* __restrict__ idx, long long row0,
    int B, float* __restrict__ slab, float* __restrict__ slab_bias) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int C = 4, IMG = 84, IMGB = C * IMG * IMG;
  constexpr int XW = 24, ROWE = 4 * XW, EST = C * IMG * ROWE;
  constexpr int NT = NW * 64, NITEM = C * IMG * 6, IPT = 2048 / NT, NS = 6;
  constexpr int TW = 32 / NW, NTAIL = 8 / NW, NP = TW * NS + NTAIL, RA = KW3_RA, RING = RA + 1;
  __shared__ __attribute__((aligned(16))) uint16_t E[2 * EST + 80];   // + the empty put slots' target
  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR): the tail's tile choice is a scalar branch
  const int kg = NW == 8 ? w >> 1 : w, t0 = NW == 8 ? 4 * (w & 1) : 0;
  const bool counts = NW == 4 || (w & 1) == 0;   // the bias sum: one wave of each k-step group
  const int G = gridDim.x;
  // column tiles: BXT (4 waves) — tile tt = (channel tt >> 1, x-phase half bx = tt & 1),
  // lane l32 = (ky = l32 >> 2, dx = l32 & 3), so a tile's whole B fragment is either
  // unshifted (bx = 0: one 8-B read per quad, no realignment) or shifted by one
  // element (bx = 1: 8-B + 4-B read, two v_alignbyte by a constant); otherwise (the
  // 8-wave form) tile tt = (channel, ky half), lane l32 = (ky & 3, kx) with a per-lane
  // shift for kx >= 4
  constexpr bool BXT = KW3_BXT && NW == 4;
  const int kx = l32 & 7, sh = 2 * (kx >> 2);
  const int lbase = BXT ? l32 * XW : ((l32 >> 3) * 4 + (kx & 3)) * XW;
  // put items: thread item j = tid + NT j (2,016 of 2,048 slots are real)
  int isrc[IPT], idst[IPT];
#pragma unroll
  for (int j = 0; j < IPT; ++j) {
    const int it = tid + NT * j, r = it / 6, g6 = it - 6 * r;
    isrc[j] = r * IMG + 16 * g6;   // >= IMGB for the empty slots: their loads read 0
    idst[j] = it < NITEM ? r * ROWE + 4 * g6 : -1;
  }
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  u32x4v raw[IPT];
  auto raw_load1 = [&](const __amdgpu_buffer_rsrc_t& rs, int j) {
    if (j < IPT - 1) {
      raw[j] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(rs, isrc[j], 0, 0));
    } else {   // the slot holding the image's last 4 bytes: dword loads (each range-checked)
#pragma unroll
      for (int k = 0; k < 4; ++k) raw[j][k] = __builtin_amdgcn_raw_buffer_load_b32(rs, isrc[j] + 4 * k, 0, 0);
    }
  };
  auto put_dx = [&](int j, int st, int dx) {   // one x-phase of item j: u8 -> bf16 (exact), de-interleaved by x mod 4
    const int d = idst[j] >= 0 ? st * EST + idst[j] : 2 * EST;
    float f[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) f[k] = (float)((raw[j][k] >> (8 * dx)) & 255u);
    const uint2 q = {__builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u),
                     __builtin_amdgcn_perm(__float_as_uint(f[3]), __float_as_uint(f[2]), 0x07060302u)};
    *reinterpret_cast<uint2*>(E + d + dx * XW) = q;
  };
  // dz of (image b, k-step s): 8 pixels 16 s + 8 h + j of channel l32
  auto dz_load1 = [&](int b, int s, f32x8& d, int j) {
    const auto rs = make_rsrc(dz1 + (size_t)b * 12800, 12800 * 4);
    const int px = 16 * s + 4 * h + (j & 3) + 8 * (j >> 2);   // quads 4 s + h, 4 s + h + 2 (see qb)
    d[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (px * 32 + l32) * 4, 0, 0));
  };
  float bacc = 0.f;
  // one pair (values 2 pr, 2 pr + 1) of split8's three-way split (the same bits)
  auto split_pair = [&](const f32x8& d, Frag3& f, int pr, bool count) {
    const float v0 = d[2 * pr], v1 = d[2 * pr + 1];
    const bf16x2 hh = __builtin_convertvector(f32x2{v0, v1}, bf16x2);
    const float r0 = v0 - (float)hh[0], r1 = v1 - (float)hh[1];
    const bf16x2 mm = __builtin_convertvector(f32x2{r0, r1}, bf16x2);
    const bf16x2 ll = __builtin_convertvector(f32x2{r0 - (float)mm[0], r1 - (float)mm[1]}, bf16x2);
    f.h[2 * pr] = hh[0]; f.h[2 * pr + 1] = hh[1];
    f.m[2 * pr] = mm[0]; f.m[2 * pr + 1] = mm[1];
    f.l[2 * pr] = ll[0]; f.l[2 * pr + 1] = ll[1];
    if (count) bacc += v0 + v1;
  };
  auto qoff = [&](int q) { const int oy = q / 5; return 4 * oy * ROWE + 4 * (q - 5 * oy); };
  // the tail (k-step 24) tile e of this wave: one of its own column tiles (NW = 4:
  // 2 w + e; NW = 8: t0 + kg)
  auto tail_tile = [&](int e) { return NW == 4 ? 2 * w + e : t0 + kg; };
  // tile p of the image's flat sequence: k-step kg + 4 (p / TW), tile t0 + p % TW (p <
  // TW NS); k-step 24, tile tail_tile(p - TW NS) (the tail)
  uint32_t braw[RING][6];
  // per-lane element offsets of the two quads of each step (lbase included): the
  // tile part of a B address is then a compile-time constant (the ds_read offset).
  // Lane half h takes quads 4 s + h and 4 s + h + 2 of the k-step (pixels 16 s + 4 h
  // .. +3, +8 .. +11; the A fragment's dz loads follow).  The 4-B tail reads are
  // 2-way bank conflicts (ds_read_b32 banks by dword mod 32; the 16 (ky, x-phase)
  // rows sit 12 dwords apart): 39 % of the LDS-active cycles
  // (profiles/r05_y_kw3_sq.json).  Reading the tail as an aligned 8-B ds_read_b64
  // (mod-64 banks: conflict-free) from an address the compiler cannot merge with the
  // head read was slower, 1.75-1.78 vs 1.51-1.53 ms (an extra address add per read)
  int qb[NS + 1][2];
#pragma unroll
  for (int i = 0; i <= NS; ++i)
#pragma unroll
    for (int k = 0; k < 2; ++k) qb[i][k] = lbase + qoff(4 * (i < NS ? kg + 4 * i : 24) + h + 2 * k);
  // the x-phase half of flat tile p (BXT; compile-time: t0 = 0 there)
  auto bx_of = [&](int p) { return p < TW * NS ? (p % TW) & 1 : (p - TW * NS) & 1; };
  auto bread = [&](const uint16_t* S, int p) {
    const int i = p < TW * NS ? p / TW : NS, tt = p < TW * NS ? t0 + p % TW : tail_tile(p - TW * NS);
    const int toff = BXT ? (tt >> 1) * IMG * ROWE : ((tt >> 1) * IMG + 4 * (tt & 1)) * ROWE;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint16_t* pp = S + toff + qb[i][k];
      const uint2 d01 = *reinterpret_cast<const uint2*>(pp);
      braw[p % RING][3 * k] = d01.x;
      braw[p % RING][3 * k + 1] = d01.y;
      if (!BXT || bx_of(p)) braw[p % RING][3 * k + 2] = *reinterpret_cast<const uint32_t*>(pp + 4);
    }
  };
  f32x16 acc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  auto mma3 = [&](int p, const Frag3& a, f32x16& c) {
    const uint32_t* r = braw[p % RING];
    bf16x8 bq;
    if (BXT && !bx_of(p)) {
      bq = __builtin_bit_cast(bf16x8, uint4{r[0], r[1], r[3], r[4]});
    } else {
      const int s2 = BXT ? 2 : sh;
      bq = __builtin_bit_cast(bf16x8, uint4{__builtin_amdgcn_alignbyte(r[1], r[0], s2),
                                            __builtin_amdgcn_alignbyte(r[2], r[1], s2),
                                            __builtin_amdgcn_alignbyte(r[4], r[3], s2),
                                            __builtin_amdgcn_alignbyte(r[5], r[4], s2)});
    }
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, bq, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, bq, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, bq, c, 0, 0, 0);
  };
  // Prefetch schedule (each slot is live only between its load and its split, so
  // the loop-carried registers stay few and the allocator does not split their live
  // ranges — a copy of an in-flight load waits for it):
  //   dz slot i (k-step kg + 4 i) is split during step i - 1 (slot 0: step 5 of the
  //   previous image); slots 4, 5 are loaded in steps 0, 1 (this image), the next
  //   image's slots 0-3 two per step in steps 2, 3 (two steps before the loop end, so
  //   the back-edge copies find the data arrived); D24 is loaded in step 1 and split
  //   in step 4;
  //   put items (converting image b + G; NW = 4: 0 | 1 | 2, 3 | 4 | 5, 6 | 7 in
  //   steps 0-5, NW = 8: 0 | 1 | - | 2 | 3 | -) are loaded four steps ahead: those
  //   put in steps 4, 5 during steps 0, 1 (image b + G), the others during steps
  //   2-5 (image b + 2G).
  f32x8 D[NS], D24;   // 8-register tuples: the allocator keeps a slot in one place
  Frag3 F[2], F24;
  int b = blockIdx.x, cur = 0;
  const auto clampb = [&](int x) { return x < B ? x : B - 1; };
  auto put_step = [](int j) {
    if constexpr (NW == 4) return j < 2 ? j : j < 4 ? 2 : j == 4 ? 3 : j < 7 ? 4 : 5;
    else return j < 2 ? j : j + 1;
  };
  if (b < B) {
    {
      const auto rs0 = make_rsrc(obs + obs_row(idx, row0, b) * (long long)IMGB, IMGB);
#pragma unroll
      for (int j = 0; j < IPT; ++j) raw_load1(rs0, j);
    }
#pragma unroll
    for (int i = 0; i < (NW == 4 ? 4 : 3); ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) dz_load1(b, kg + 4 * i, D[i], j);
    wait_vm0();
#pragma unroll
    for (int j = 0; j < IPT; ++j)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) put_dx(j, 0, dx);
    {
      const auto rs1 = make_rsrc(obs + obs_row(idx, row0, clampb(b + G)) * (long long)IMGB, IMGB);
#pragma unroll
      for (int j = 0; j < IPT; ++j)
        if (put_step(j) <= 3) raw_load1(rs1, j);
    }
#pragma unroll
    for (int pr = 0; pr < 4; ++pr) split_pair(D[0], F[0], pr, counts);
    // nothing in flight at the loop entry: the waitcnt pass merges the entry and the
    // back-edge states at the loop head, and prologue loads with few younger loads
    // behind them would cap every iteration's waits (vmcnt(1) at step 0)
    wait_vm0();
    lds_barrier();
#pragma unroll
    for (int p = 0; p < RA; ++p) bread(E, p);
  }
  for (; b < B; b += G) {
    const uint16_t* Sc = E + cur * EST;
    const int bn = clampb(b + G);
    const auto rs1 = make_rsrc(obs + obs_row(idx, row0, bn) * (long long)IMGB, IMGB);
    const auto rs2 = make_rsrc(obs + obs_row(idx, row0, clampb(b + 2 * G)) * (long long)IMGB, IMGB);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      int ja = -1, jb = -1;   // the step's put items
#pragma unroll
      for (int j = 0; j < IPT; ++j)
        if (put_step(j) == i) {
          if (ja < 0) ja = j;
          else jb = j;
        }
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int p = TW * i + t;
        if (p + RA < NP) bread(Sc, p + RA);
#if KW3_FENCE
        __builtin_amdgcn_sched_barrier(0);   // the read-ahead stays ahead of this tile's MFMAs
#endif
        mma3(p, F[i & 1], acc[t]);
        // filler work, sliced evenly over the step's tiles (a tile's MFMAs and its
        // slice share one scheduling region between the fences): pairs of the next
        // step's split (and of the tail's in step 4), the dz slot loads, the x-phases
        // of the step's put item(s), then the raw loads four steps ahead
        if (t < 4) {
          if (i + 1 < NS) split_pair(D[i + 1], F[(i + 1) & 1], t, counts);
          else split_pair(D[0], F[0], t, counts && b + G < B);
        }
        if (i == 4 && t >= TW - 4) split_pair(D24, F24, t - (TW - 4), w == 0);
#pragma unroll
        for (int u = 0; u < 8 / TW; ++u) {
          const int jl = (8 / TW) * t + u;   // load jl of the slot's 8
          if constexpr (NW == 4) {
            if (i < 2) dz_load1(b, kg + 4 * (4 + i), D[4 + i], jl);
            if (i == 2 || i == 3) {
              dz_load1(bn, kg + 4 * (2 * (i - 2)), D[2 * (i - 2)], jl);
              dz_load1(bn, kg + 4 * (2 * (i - 2) + 1), D[2 * (i - 2) + 1], jl);
            }
            if (i == 1) dz_load1(b, 24, D24, jl);
          } else {   // two waves per SIMD: shorter distances — slots 3, 4, 5 (this image)
                     // in steps 0-2, the next image's 0 in step 3, 1 and 2 in step 4
            if (i < 3) dz_load1(b, kg + 4 * (3 + i), D[3 + i], jl);
            if (i == 3) dz_load1(bn, kg, D[0], jl);
            if (i == 4) {
              dz_load1(bn, kg + 4, D[1], jl);
              dz_load1(bn, kg + 8, D[2], jl);
            }
            if (i == 2) dz_load1(b, 24, D24, jl);
          }
        }
        if (ja >= 0) {
          if (jb < 0) {
            if (t < 4) put_dx(ja, cur ^ 1, t);
          } else {
            put_dx(t < 4 ? ja : jb, cur ^ 1, t & 3);
          }
        }
        if (t == TW - 1) {
#pragma unroll
          for (int jj = 0; jj < IPT; ++jj) {
            if (i < 2 && put_step(jj) == i + 4) raw_load1(rs1, jj);
            if (i >= 2 && put_step(jj) == i - 2) raw_load1(rs2, jj);
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < NTAIL; ++e) {   // the tail: tile tail_tile(e) of k-step 24
      const int p = TW * NS + e;
      if (p + RA < NP) bread(Sc, p + RA);
#pragma unroll
      for (int t = 0; t < TW; ++t)
        if (t0 + t == tail_tile(e)) mma3(p, F24, acc[t]);
    }
    lds_barrier();   // E[cur ^ 1] complete, E[cur] consumed
    cur ^= 1;
    if (b + G < B) {
#pragma unroll
      for (int p = 0; p < RA; ++p) bread(E + cur * EST, p);
    }
  }
  wait_vm0();
  __syncthreads();
  // the k-step groups' partial gradients summed in a fixed order (per column half)
  float* X = reinterpret_cast<float*>(E);
  const int slot = NW == 8 ? (w & 1) : 0;
#pragma unroll
  for (int half = 2; half >= 1; half >>= 1) {
    if (kg >= half && kg < 2 * half) {
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[((((kg - half) * 2 + slot) * TW + t) * 16 + r) * 64 + lane] = acc[t][r];
    }
    __syncthreads();
    if (kg < half) {
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += X[(((kg * 2 + slot) * TW + t) * 16 + r) * 64 + lane];
    }
    __syncthreads();
  }
  float* out = slab + (size_t)blockIdx.x * 32 * 256;
  if (kg == 0) {
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int n = BXT ? 64 * (t >> 1) + 8 * (l32 >> 2) + 4 * (t & 1) + (l32 & 3) : 32 * (t0 + t) + l32;
        out[co * 256 + n] = acc[t][r];
      }
  }
  X[tid] = bacc;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < NW; ++v) t += X[v * 64 + tid] + X[v * 64 + 32 + tid];
    slab_bias[(size_t)blockIdx.x * 32 + tid] = t;
  }
}

}  // namespace

int conv1_wgrad_kw3(const float* dz1, const uint8_t* obs, const int64_t* idx, long long row0, int B, int Z,
                    float* slab, float* slab_bias, void* stream, int nw) {
  if (B <= 0 || Z <= 0) return 0;
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin("conv1_wgrad_u8", st, &slot);
  if (nw == 8) conv1_wgrad_kw3_kernel<8><<<Z, 512, 0, st>>>(dz1, obs, idx, row0, B, slab, slab_bias);
  else conv1_wgrad_kw3_kernel<4><<<Z, 256, 0, st>>>(dz1, obs, idx, row0, B, slab, slab_bias);
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_wgrad_kw3_kernel");
  return 0;
}

// conv1 weight gradient of u8 observations (C = 4) with the k-split kernel: slab [Z][32][256]
// (integer-scaled: reduce with 1/255) and bias partials [Z][32]; called by ppo_conv1_wgrad (tune 8)
int conv1_wgrad_kw(const float* dz1, const uint8_t* obs, const int64_t* idx, long long row0, int B, int Z,
                   float* slab, float* slab_bias, void* stream) {
  if (B <= 0 || Z <= 0) return 0;
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin("conv1_wgrad_u8", st, &slot);
  conv1_wgrad_kw2_kernel<8><<<Z, 512, 0, st>>>(dz1, obs, idx, row0, B, slab, slab_bias);
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_wgrad_kw2_kernel");
  return 0;
}
