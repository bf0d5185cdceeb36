// conv1 forward on raw u8 RGB frames by the affine fold of the env chain
// (ppo_tune_set("rgb_aff", 1), default; round 4).
//
// The OTC v7 observation chain (T/make_env.py:411-413) feeds conv1 (model.py:177)
//   X_c[y][x] = (u[y][x][c] - m[y][x][c]) / s                     c = 0, 1, 2
//   X_3[y][x] = 0.299 X_0[x][y] + 0.587 X_1[x][y] + 0.114 X_2[x][y] (grey, transposed)
// (NormalizeWrapper, T/sohojoe_wrappers.py:958-991; FrameStackMono(2), :563-638).
// Both are affine in the raw bytes u, so
//   conv1(X)[co][oy][ox] = b[co] + Σ_c Σ_(ky,kx) W[co][c][ky][kx] X_c[4oy+ky][4ox+kx]
//                         + Σ_c Σ_(r,q) k_c W[co][3][q][r] X_c[4ox+r][4oy+q]
//                       = rs · Σ_k Weff[co][k] u_k(oy, ox) + Mb[(oy, ox)][co]
// with K = 384: k < 192 the direct patch of the three colour planes at (4oy, 4ox),
// k >= 192 the patch at the transposed origin (4ox, 4oy) with the grey-folded,
// transposed weights; rs = 1/s and the map Mb = b - rs Σ_k Weff m_k (the means'
// share, fixed between optimizer steps) are computed per call by a small prep
// kernel.  The raw bytes are exact in bf16, so the MFMA part is the u8 kernels'
// exact arithmetic (three weight parts, products exact, fp32 accumulation) over
// 1.5x their K — no per-element decode (the bit-exact fused decode of conv1f.hip,
// which redoes the float64 normalisation on every read of a frame, stays as
// rgb_aff 0).  The results differ from the decode chain at fp32 rounding level
// (the fl32 of each normalised element and of the grey sums are not formed;
// tests/test_obs_paths.py compares both against float64).  Not for the raw mode
// (no normaliser, s = 1): FrameStackMono truncates that grey plane to u8 — not
// affine — so it keeps the decode kernel.
//
// Kernel: one persistent block (8 waves) per CU walks images.  The weights' three
// bf16 parts sit in LDS (split once per block, 75,264 B: in registers they would
// need 144 VGPRs and spill), the frame's three colour planes as bf16 [c][84][84]
// (two stages, 84,672 B); item i of
// a frame (pixels 16i .. 16i+15, 48 B, i < 441) is loaded by thread i one image
// ahead and de-interleaved into the planes.  Wave w: output channels 16 (w & 1)
// + [0, 16), row tiles {w >> 1, (w >> 1) + 4, ...} of 16 output pixels; k-step s
// (12 of 32): s < 6 plane s >> 1, patch rows 4 (s & 1) + g of the direct origin;
// s >= 6 plane (s - 6) >> 1, patch rows 4 ((s - 6) & 1) + g of the transposed
// origin — every pixel fragment is 8 consecutive bf16 of one plane row (two
// 8-B LDS reads), as in the u8 kernel.
#include <mutex>

#include "igemm_x9.h"

namespace {

constexpr int RA_IMG = 84, RA_NPX = RA_IMG * RA_IMG, RA_FB = RA_NPX * 3;   // 21,168 B per frame
constexpr int RA_K = 384, RA_KS = RA_K / 32, RA_NT = 7, RA_ITEMS = RA_NPX / 16;   // 441 items of 16 px

// Weff [32][384] and Mb [400][32] (see the header)
__global__ __launch_bounds__(512) void rgbaff_prep_kernel(const float* __restrict__ w1, const float* __restrict__ b1,
                                                          const float* __restrict__ mean, double rs,
                                                          float* __restrict__ weff, float* __restrict__ mb) {
  const int co = blockIdx.x, tid = threadIdx.x;
  __shared__ float we[RA_K];
  const float kg[3] = {0.299f, 0.587f, 0.114f};
  for (int k = tid; k < RA_K; k += 512) {
    float v;
    if (k < 192) {
      const int c = k >> 6, ky = (k >> 3) & 7, kx = k & 7;
      v = w1[((co * 4 + c) * 8 + ky) * 8 + kx];
    } else {
      const int kk = k - 192, c = kk >> 6, r = (kk >> 3) & 7, q = kk & 7;
      v = kg[c] * w1[((co * 4 + 3) * 8 + q) * 8 + r];
    }
    we[k] = v;
    weff[co * RA_K + k] = v;
  }
  __syncthreads();
  if (tid < 400) {
    const int oy = tid / 20, ox = tid - 20 * oy;
    double acc = 0.0;
    if (mean) {
      for (int k = 0; k < RA_K; ++k) {
        int y, x, c;
        if (k < 192) {
          c = k >> 6;
          y = 4 * oy + ((k >> 3) & 7);
          x = 4 * ox + (k & 7);
        } else {
          const int kk = k - 192;
          c = kk >> 6;
          y = 4 * ox + ((kk >> 3) & 7);
          x = 4 * oy + (kk & 7);
        }
        acc += (double)we[k] * (double)mean[(y * RA_IMG + x) * 3 + c];
      }
    }
    mb[tid * 32 + co] = (float)((double)b1[co] - acc * rs);
  }
}

template <bool MASK, int NPW>
__global__ __launch_bounds__(512) void conv1_fwd_rgbaff_kernel(const uint8_t* __restrict__ frames,
                                                               const int64_t* __restrict__ idx, long long row0, int B,
                                                               const float* __restrict__ weff,
                                                               const float* __restrict__ mb, float rs,
                                                               float* __restrict__ out, uint16_t* __restrict__ mbits) {
  __shared__ __attribute__((aligned(16))) uint16_t img[2][3 * RA_NPX];   // 84,672 B
  // the weights' bf16 parts [part][co][k] (rows padded to 392: 784 B, so the 16
  // columns of a fragment read start on distinct 16-B bank slots); 75,264 B
  constexpr int WR = RA_K + 8;
  __shared__ __attribute__((aligned(16))) uint16_t Wl[3 * 32 * WR];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, rq = wave >> 1, ntile = rq == 0 ? 7 : 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int col = ct * 16 + i16;
  for (int i = tid; i < 32 * RA_K; i += 512) {   // split once per block
    const int co = i / RA_K, k = i - co * RA_K;
    uint32_t h, m, l;
    if constexpr (NPW == 1) {
      h = bf16_rne_bits(weff[i]);
      m = l = 0;
    } else {
      split_bf16x3(weff[i], h, m, l);
    }
    Wl[co * WR + k] = (uint16_t)h;
    Wl[32 * WR + co * WR + k] = (uint16_t)m;
    Wl[64 * WR + co * WR + k] = (uint16_t)l;
  }
  uint4 stage[3];
  auto fetch = [&](int b) {   // item tid (48 B); threads past the items read out of range (0)
    const auto rsrc = make_rsrc(frames + obs_row(idx, row0, b) * (long long)RA_FB, RA_FB);
    const int off = tid < RA_ITEMS ? 48 * tid : 0x7fffff00;
#pragma unroll
    for (int j = 0; j < 3; ++j)
      stage[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 16 * j, 0, 0));
  };
  auto put = [&](int buf) {   // HWC bytes -> the three bf16 planes (exact), 16 pixels per item
    if (tid >= RA_ITEMS) return;
    const uint32_t w[12] = {stage[0].x, stage[0].y, stage[0].z, stage[0].w, stage[1].x, stage[1].y,
                            stage[1].z, stage[1].w, stage[2].x, stage[2].y, stage[2].z, stage[2].w};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint32_t o[8];
#pragma unroll
      for (int pq = 0; pq < 8; ++pq) {
        const int j0 = 3 * (2 * pq) + c, j1 = j0 + 3;
        const float f0 = (float)((w[j0 >> 2] >> (8 * (j0 & 3))) & 255u);
        const float f1 = (float)((w[j1 >> 2] >> (8 * (j1 & 3))) & 255u);
        o[pq] = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
      }
      uint4* d = reinterpret_cast<uint4*>(img[buf] + c * RA_NPX + 16 * tid);
      d[0] = uint4{o[0], o[1], o[2], o[3]};
      d[1] = uint4{o[4], o[5], o[6], o[7]};
    }
  };
  int pix[RA_NT], pixT[RA_NT];   // direct / transposed patch origin of this lane's row, per row tile
#pragma unroll
  for (int t = 0; t < RA_NT; ++t) {
    const int row = min((rq + 4 * t) * 16 + i16, 399), oy = row / 20, ox = row - oy * 20;
    pix[t] = oy * (4 * RA_IMG) + ox * 4;
    pixT[t] = ox * (4 * RA_IMG) + oy * 4;
  }
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
    put(0);
    if (b + G < B) fetch(b + G);
  }
  __syncthreads();
  for (; b < B; b += G) {
    if (b + G < B) put(cur ^ 1);   // read two iterations ago; the last barrier retired it
    if (b + 2 * G < B) fetch(b + 2 * G);
    const uint16_t* I = img[cur];
    f32x4 acc[RA_NT];
#pragma unroll
    for (int t = 0; t < RA_NT; ++t) acc[t] = zero4();
#pragma unroll
    for (int s = 0; s < RA_KS; ++s) {
      const int sp = s < 6 ? s : s - 6;
      const uint16_t* Is = I + (sp >> 1) * RA_NPX + (4 * (sp & 1) + g) * RA_IMG;
      bf16x8 a[RA_NT];
#pragma unroll
      for (int t = 0; t < RA_NT; ++t)
        if (t < ntile) {
          const uint2* p2 = reinterpret_cast<const uint2*>(Is + (s < 6 ? pix[t] : pixT[t]));   // 8-B aligned
          const uint2 lo = p2[0], hi = p2[1];
          a[t] = __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y});
        }
      bf16x8 wf[NPW];   // B[k][n] = Weff[n][k], this k-step's parts
#pragma unroll
      for (int part = 0; part < NPW; ++part)
        wf[part] = *reinterpret_cast<const bf16x8*>(Wl + (part * 32 + col) * WR + 32 * s + 8 * g);
#pragma unroll
      for (int part = 0; part < NPW; ++part)
#pragma unroll
        for (int t = 0; t < RA_NT; ++t)
          if (t < ntile) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t], wf[part], acc[t], 0, 0, 0);
    }
    float* o = out + (size_t)b * (400 * 32) + col;
#pragma unroll
    for (int t = 0; t < RA_NT; ++t)
      if (t < ntile) {
        const int rt = rq + 4 * t;
        uint64_t bal[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rt * 16 + 4 * g + r;
          const float v = fmaxf(acc[t][r] * rs + mb[row * 32 + col], 0.f);
          o[row * 32] = v;
          if constexpr (MASK) bal[r] = __builtin_amdgcn_ballot_w64(v > 0.f);
        }
        if constexpr (MASK) {   // as the u8 kernel: lane j < 16 stores pixel 16 rt + j's 16 channel bits
          if (lane < 16) {
            const int r = lane & 3, gg = lane >> 2;
            const uint64_t bsel = r == 0 ? bal[0] : r == 1 ? bal[1] : r == 2 ? bal[2] : bal[3];
            mbits[((size_t)b * 400 + rt * 16 + lane) * 2 + ct] = (uint16_t)(bsel >> (16 * gg));
          }
        }
      }
    __syncthreads();   // every wave is done with img[cur]; img[cur ^ 1] is complete
    cur ^= 1;
  }
}

// ---------------------------------------------------------------------------
// Weight gradient by the same fold.  With X_c = rs (u_c - m_c):
//   dW[co][c][ky][kx] = rs (G[co][c][ky][kx] - Gm[...])                 c < 3
//   dW[co][3][ky][kx] = rs Σ_c k_c (GT[co][c][kx][ky] - GmT[...])
//   G  = Σ_(b,p) dz[b][p][co] u_c[4oy+ky][4ox+kx],  GT the same at the transposed
//   origin (4ox + r, 4oy + q);  Gm / GmT the same sums over the means with
//   D[co][p] = Σ_b dz[b][p][co] in place of dz (the means do not depend on b).
// G and GT are two passes of the u8 k-split kernel (conv1w.hip kw2: the raw frame
// by LDS-DMA, phase rows converted once per image, two E stages, dz straight from
// HBM and split in registers) over the three colour planes of the frame (TRANS:
// of its transpose, u^T[y][x] = u[x][y]) — 6 column tiles of 32 instead of 8;
// the direct pass also sums D per block (its dz values are in registers anyway)
// into a [Z][32][400] scratch.  Each pass writes its columns of the block's slab
// already scaled by rs (direct: n < 192; TRANS: the grey channel's 64 columns,
// summed over c with k_c and transposed) and the direct pass the bias partials;
// rgbaff_wfinal subtracts the means' share from slab 0.  Slab format and bias as
// every conv1 wgrad (the engine's ppo_wgrad_reduce sums the Z slabs, scale 1).
template <bool TRANS>
__global__ __launch_bounds__(512) void conv1_wgrad_rgbaff_kernel(const float* __restrict__ dz1,
                                                                 const uint8_t* __restrict__ frames,
                                                                 const int64_t* __restrict__ idx, long long row0,
                                                                 int B, float rs, float* __restrict__ slab,
                                                                 float* __restrict__ slab_bias,
                                                                 float* __restrict__ dsum) {
  constexpr int NW = 8, C = 3, IMG = RA_IMG, NTL = 2 * C;   // 6 column tiles of 32
  constexpr int XW = 24, ROWE = 4 * XW, EST = C * IMG * ROWE;  // 24,192 elements per stage
  constexpr int NITEM = IMG * 6, NPC = 21, RAWB = NPC * 1024;  // items (y, 16-x group); raw pieces
  __shared__ __attribute__((aligned(16))) uint16_t E[2 * EST + RAWB / 2];   // 118,272 B
  uint8_t* const RAW = reinterpret_cast<uint8_t*>(E + 2 * EST);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int G = gridDim.x;
  const int kx = l32 & 7, dxl = kx & 3, sh = 2 * (kx >> 2);
  const int lbase = ((l32 >> 3) * 4 + dxl) * XW;
  const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(RAW);
  auto dma_raw = [&](int b) {   // pieces wave + 8 i (i < 3), clamped: harmless duplicates / tail
    const uint8_t* img = frames + obs_row(idx, row0, b) * (long long)RA_FB;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int pc = min(wave + 8 * i, NPC - 1);
      const int off = min(pc * 1024 + lane * 16, RA_FB - 16);
      glds16(img + off, __builtin_amdgcn_readfirstlane(raw_lds + pc * 1024));
    }
  };
  // RAW (HWC bytes) -> E[st][c][y][dx][X] = plane value at (y, 4X + dx), bf16 (exact);
  // the plane is u_c (direct) or u_c^T (TRANS); x >= 84 (never read) clamped
  auto put = [&](int st) {
    uint16_t* S = E + st * EST;
    if (tid >= NITEM) return;
    const int y = tid / 6, g6 = tid - 6 * y;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      float f[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int x = min(16 * g6 + j, IMG - 1);
        const int byte = TRANS ? (x * IMG + y) * 3 + c : (y * IMG + x) * 3 + c;
        f[j] = (float)RAW[byte];
      }
      uint16_t* dp = S + (c * IMG + y) * ROWE + 4 * g6;
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {   // X = 4 g6 + jj: x = 16 g6 + 4 jj + dx
        const uint2 q = {__builtin_amdgcn_perm(__float_as_uint(f[4 + dx]), __float_as_uint(f[dx]), 0x07060302u),
                         __builtin_amdgcn_perm(__float_as_uint(f[12 + dx]), __float_as_uint(f[8 + dx]), 0x07060302u)};
        *reinterpret_cast<uint2*>(dp + dx * XW) = q;
      }
    }
  };
  f32x16 acc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bacc = 0.f;
  float dacc[4][8];   // !TRANS: D sums of this lane's pixels per k-step slot (A, B, C, D)
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) dacc[q][j] = 0.f;
  auto dz_load = [&](int b, int s, float (&d)[8]) {
    const auto rsc = make_rsrc(dz1 + (size_t)b * 12800, 12800 * 4);
    const int o = ((16 * s + 8 * h) * 32 + l32) * 4;
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsc, o + 128 * j, 0, 0));
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
    for (int tt = 0; tt < NTL; ++tt) {
      if (tt < t0 || tt >= t1) continue;
      const bf16x8 bq = bfrag(S, tt, o0, o1);
      acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, bq, acc[tt], 0, 0, 0);
      acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, bq, acc[tt], 0, 0, 0);
      acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, bq, acc[tt], 0, 0, 0);
    }
  };
  auto add8 = [&](const float (&d)[8], int slot) {
    if constexpr (!TRANS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bacc += d[j];
        dacc[slot][j] += d[j];
      }
    }
  };
  int b = blockIdx.x, cur = 0;
  float dA[8], dB[8], dC[8], dD[8];
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
    kstep(S, wave, dA, 0, NTL);
    add8(dA, 0);
    dz_load(b, 24, dD);
    kstep(S, wave + 8, dB, 0, NTL);
    add8(dB, 1);
    if (nxt) {
      // raw(b + G) is older than dB's loads, which k-step B waited for; the explicit wait
      // (dC, dD may stay in flight) makes the order independent of the compiler's waits
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      lds_barrier();   // Y: every wave's pieces of raw(b + G) are in LDS
      put(cur ^ 1);
      lds_barrier();   // Z: raw consumed, E[cur ^ 1] complete
      dz_load(b + G, wave, dA);
      dz_load(b + G, wave + 8, dB);
      if (b + 2 * G < B) dma_raw(b + 2 * G);
    }
    kstep(S, wave + 16, dC, 0, NTL);
    add8(dC, 2);
    kstep(S, 24, dD, wave, wave + 1);     // k-step 24: tile `wave` (waves 6, 7: none; D and bias: wave 0)
    if (wave == 0) add8(dD, 3);
    cur ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // D partial: lane (l32, h) of wave w, slot q: pixels 16 s_q + 8 h + j of channel l32
  if constexpr (!TRANS) {
    float* dp = dsum + (size_t)blockIdx.x * (32 * 400) + l32 * 400;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q == 3 && wave != 0) continue;
      const int s = q == 0 ? wave : q == 1 ? wave + 8 : q == 2 ? wave + 16 : 24;
#pragma unroll
      for (int j = 0; j < 8; ++j) dp[16 * s + 8 * h + j] = dacc[q][j];
    }
  }
  // fixed-order sum of the eight waves' partials (as kw2), three tiles at a time
  float* X = reinterpret_cast<float*>(E);
#pragma unroll
  for (int half = 4; half >= 1; half >>= 1)
#pragma unroll
    for (int t0 = 0; t0 < NTL; t0 += 3) {
      if (wave >= half && wave < 2 * half) {
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) X[(((wave - half) * 3 + t) * 16 + r) * 64 + lane] = acc[t0 + t][r];
      }
      __syncthreads();
      if (wave < half) {
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t0 + t][r] += X[((wave * 3 + t) * 16 + r) * 64 + lane];
      }
      __syncthreads();
    }
  float* out = slab + (size_t)blockIdx.x * 32 * 256;
  if (wave == 0) {
    if constexpr (!TRANS) {   // columns n = 32 t + l32 = 64 c + 8 ky + kx, c < 3
#pragma unroll
      for (int t = 0; t < NTL; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
          out[co * 256 + 32 * t + l32] = rs * acc[t][r];
        }
    } else {   // the grey channel: column (ky', kx') of tile 2c + hh reads u_c[4ox + kx'][4oy + ky'],
      // the patch of W_3[ky'][kx'] (r = kx', q = ky'): dW3 column 192 + 8 ky' + kx' = 192 + 32 hh + l32
      const float kg[3] = {0.299f, 0.587f, 0.114f};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
          const float v = kg[0] * acc[hh][r] + kg[1] * acc[2 + hh][r] + kg[2] * acc[4 + hh][r];
          out[co * 256 + 192 + 32 * hh + l32] = rs * v;
        }
    }
  }
  if constexpr (!TRANS) {
    X[tid] = bacc;
    __syncthreads();
    if (tid < 32) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += X[w * 64 + tid] + X[w * 64 + 32 + tid];
      slab_bias[(size_t)blockIdx.x * 32 + tid] = t;
    }
  }
}

// slab 0 -= rs (Gm, Σ_c k_c GmT transposed): the means' share, D = Σ_z dsum[z]
__global__ __launch_bounds__(512) void rgbaff_wfinal_kernel(const float* __restrict__ dsum, int Z,
                                                            const float* __restrict__ mean, double rs,
                                                            float* __restrict__ slab) {
  const int co = blockIdx.x, tid = threadIdx.x;
  __shared__ float Dl[400];
  __shared__ double Gm[RA_K];
  if (tid < 400) {
    float t = 0.f;
    for (int z = 0; z < Z; ++z) t += dsum[((size_t)z * 32 + co) * 400 + tid];
    Dl[tid] = t;
  }
  __syncthreads();
  if (tid < RA_K) {
    double acc = 0.0;
    for (int p = 0; p < 400; ++p) {
      const int oy = p / 20, ox = p - 20 * oy;
      int y, x, c;
      if (tid < 192) {
        c = tid >> 6;
        y = 4 * oy + ((tid >> 3) & 7);
        x = 4 * ox + (tid & 7);
      } else {
        const int kk = tid - 192;
        c = kk >> 6;
        y = 4 * ox + ((kk >> 3) & 7);
        x = 4 * oy + (kk & 7);
      }
      acc += (double)Dl[p] * (double)mean[(y * RA_IMG + x) * 3 + c];
    }
    Gm[tid] = acc;
  }
  __syncthreads();
  float* out = slab + co * 256;
  if (tid < 192) {
    out[tid] -= (float)(rs * Gm[tid]);
  } else if (tid < 256) {   // column 192 + 8 ky + kx <- GmT[c][r = kx][q = ky]
    const int n = tid - 192, ky = n >> 3, kx = n & 7;
    const double v = 0.299f * Gm[192 + 8 * kx + ky] + 0.587f * Gm[256 + 8 * kx + ky] + 0.114f * Gm[320 + 8 * kx + ky];
    out[tid] -= (float)(rs * v);
  }
}

// Weff / Mb workspace per (device, stream): launches in flight on different
// streams never share it.  Grow-only list; the buffers live for the process.
struct AffWs {
  int dev;
  hipStream_t stream;
  float* buf;
  float* dsum;   // [zcap][32][400] (the weight gradient's per-block D sums)
  int zcap;
};
static std::mutex g_aff_mu;
static AffWs g_aff[64];
static int g_naff = 0;

static float* aff_ws(hipStream_t st) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_aff_mu);
  for (int i = 0; i < g_naff; ++i)
    if (g_aff[i].dev == dev && g_aff[i].stream == st) return g_aff[i].buf;
  if (g_naff == 64) return nullptr;
  float* p = nullptr;
  if (hipMalloc(&p, (size_t)(32 * RA_K + 400 * 32) * sizeof(float)) != hipSuccess) return nullptr;
  g_aff[g_naff++] = AffWs{dev, st, p, nullptr, 0};
  return p;
}

static float* aff_dsum(hipStream_t st, int Z) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (!aff_ws(st)) return nullptr;
  std::lock_guard<std::mutex> lk(g_aff_mu);
  for (int i = 0; i < g_naff; ++i)
    if (g_aff[i].dev == dev && g_aff[i].stream == st) {
      AffWs& w = g_aff[i];
      if (Z > w.zcap) {
        if (w.dsum) {
          if (hipStreamSynchronize(st) != hipSuccess) return nullptr;   // its launches are done
          (void)hipFree(w.dsum);
        }
        const int cap = Z > 512 ? Z : 512;
        w.dsum = nullptr;
        w.zcap = 0;
        if (hipMalloc(&w.dsum, (size_t)cap * 32 * 400 * sizeof(float)) != hipSuccess) return nullptr;
        w.zcap = cap;
      }
      return w.dsum;
    }
  return nullptr;
}

}  // namespace

// the affine-folded forward (called by ppo_conv1_fwd_rgb when rgb_aff is on and the
// mode is affine: a normaliser, or s != 1); mbits nullable
int conv1_fwd_rgb_affine(const uint8_t* frames, const int64_t* idx, long long row0, int B, const float* mean,
                         double stdv, const float* w1, const float* b1, float* out, uint32_t* mbits, void* stream) {
  if (B <= 0) return 0;
  hipStream_t st = as_stream(stream);
  float* ws = aff_ws(st);
  if (!ws) {
    ppo_set_error("ppo_conv1_fwd_rgb: workspace allocation failed");
    return PPO_EARG;
  }
  float* weff = ws;
  float* mb = ws + 32 * RA_K;
  const double rs = 1.0 / stdv;
  rgbaff_prep_kernel<<<32, 512, 0, st>>>(w1, b1, mean, rs, weff, mb);
  PPO_LAUNCH_CHECK("rgbaff_prep_kernel");
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || n_cu <= 0)
    n_cu = 256;
  const unsigned nb = (unsigned)(B < n_cu ? B : n_cu);
  const int np = ppo_tune_get("products");
  uint16_t* mb16 = reinterpret_cast<uint16_t*>(mbits);
  int slot;
  const bool prof = ppo_prof_begin("conv1_fwd_rgb", st, &slot);
  if (np == 1) {
    if (mbits) conv1_fwd_rgbaff_kernel<true, 1><<<nb, 512, 0, st>>>(frames, idx, row0, B, weff, mb, (float)rs, out, mb16);
    else conv1_fwd_rgbaff_kernel<false, 1><<<nb, 512, 0, st>>>(frames, idx, row0, B, weff, mb, (float)rs, out, nullptr);
  } else {
    if (mbits) conv1_fwd_rgbaff_kernel<true, 3><<<nb, 512, 0, st>>>(frames, idx, row0, B, weff, mb, (float)rs, out, mb16);
    else conv1_fwd_rgbaff_kernel<false, 3><<<nb, 512, 0, st>>>(frames, idx, row0, B, weff, mb, (float)rs, out, nullptr);
  }
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_fwd_rgbaff_kernel");
  return 0;
}

// the affine-folded weight gradient (called by ppo_conv1_wgrad_rgb under the same
// conditions as the forward): slab [Z][32][256] (rs-scaled) and bias partials [Z][32]
int conv1_wgrad_rgb_affine(const float* dz1, const uint8_t* frames, const int64_t* idx, long long row0, int B,
                           const float* mean, double stdv, int Z, float* slab, float* slab_bias, void* stream) {
  if (B <= 0 || Z <= 0) return 0;
  hipStream_t st = as_stream(stream);
  float* dsum = aff_dsum(st, Z);
  if (!dsum) {
    ppo_set_error("ppo_conv1_wgrad_rgb: workspace allocation failed");
    return PPO_EARG;
  }
  const double rs = 1.0 / stdv;
  int slot;
  const bool prof = ppo_prof_begin("conv1_wgrad_rgb", st, &slot);
  conv1_wgrad_rgbaff_kernel<false><<<Z, 512, 0, st>>>(dz1, frames, idx, row0, B, (float)rs, slab, slab_bias, dsum);
  conv1_wgrad_rgbaff_kernel<true><<<Z, 512, 0, st>>>(dz1, frames, idx, row0, B, (float)rs, slab, slab_bias, dsum);
  if (mean) rgbaff_wfinal_kernel<<<32, 512, 0, st>>>(dsum, Z, mean, rs, slab);
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 400 * 32 * 256);
  PPO_LAUNCH_CHECK("conv1_wgrad_rgbaff_kernel");
  return 0;
}
