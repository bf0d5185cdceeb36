// conv1 weight gradient on u8 observations, k-split over waves (round 4;
// ppo_tune_set("conv1_wgrad", 8), the default):
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

}  // namespace

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
