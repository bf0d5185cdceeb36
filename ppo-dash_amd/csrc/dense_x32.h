// dense_x32.h — the CNNBase fc GEMMs (model.py:181, Linear(32*7*7, H) + ReLU, and
// its input gradient) on v_mfma_f32_32x32x16_bf16, fp32-exact by the split of
// igemm_x9.h, included by gemm.hip.
//
//   out[m][n] = epi( Σ_k x[m][k] · W[n][k] )        x fp32 [M][K], W [N][K]
//
// Weights are the MFMA A operand (rows n, the pre-split bf16 planes of
// ppo_pack_weights), activations the B operand (columns m, fp32, split into
// hi / mid / lo at fragment-read time): the accumulator lane then holds four
// consecutive n of one m.  Block tile 256 n x 128 m, 8 waves of 128 n x 32 m (4
// tiles of 32 x 32, 64 accumulator VGPRs: each split activation fragment feeds 4 x NP MFMAs), BK 32, two LDS stages of 64 KB
// filled by LDS-DMA (global_load_lds_dwordx4: no staging registers, no VALU,
// no ds_write) — the generic tile core (igemm_x9.h) stages through registers,
// splits with every wave and holds 128 x 128 tiles, so the fc input was read 4x.
// Here x is read N / 256 times (twice for fc forward, H = 512).
//   * LDS slots (16 B): weight plane p row r chunk q at p * 1024 + 4 r +
//     (q ^ ((r >> 2) & 3)); activation row r chunk c at 3072 + 8 r + (c ^ ((r >> 1)
//     & 7)): the four 16-lane groups of a ds_read_b128 hit 16 distinct slots of a
//     256-B bank row.  A DMA wave-instruction fills 64 consecutive slots, so the
//     swizzle is applied to the source addresses.
//   * Epilogue through LDS (the stages are free after the last k-step): the
//     128 x 256 fp32 tile, 16-B unit c of row m at c ^ (m & 63), then every wave
//     stores whole 1-KB rows (coalesced), applying bias + ReLU or the ReLU mask
//     of the layer below.
// XCD-aware tile order: xcd_remap makes the tiles of one XCD contiguous and the
// tile index is n-block-major, so an XCD streams the weight slice of one or two
// n-blocks from its own L2.
#pragma once

namespace {

enum { DX_BIAS_RELU = 0, DX_MASK = 1 };

struct DenseX32Args {
  const uint16_t* wpl; long long wps;   // weight plane p, row n: wpl + p * wps + n * K (bf16)
  const float* x; long long ldx;        // activations [M][K], row stride ldx floats
  float* out; long long ldo;            // [M][ldo]
  const float* bias;                    // DX_BIAS_RELU: out = relu(v + bias[n])
  const float* act; long long ldact;    // DX_MASK: out = act[m][n] > 0 ? v : 0
  int M, N, K, mblocks;
  int dbg;   // timing anatomy only (wrong results): 4 no epilogue, 8 no DMA, 16 all blocks on tile 0
};

constexpr int DX_BN = 256, DX_BM = 128;

// 16-B slot of chunk q of row r in a tile of Q chunks per row, XOR-swizzled so the
// 16-lane groups of a ds_read_b128 (16 rows, one chunk) hit 16 distinct slots
template <int Q>
__device__ __forceinline__ int dx_slot(int row, int q) {
  if constexpr (Q == 8) return 8 * row + (q ^ ((row >> 1) & 7));
  else if constexpr (Q == 4) return 4 * row + (q ^ ((row >> 2) & 3));
  else return 2 * row + (q ^ ((row >> 3) & 1));
}
__device__ __forceinline__ __attribute__((address_space(3))) void* dx_lds(const void* p) {
  return reinterpret_cast<__attribute__((address_space(3))) void*>(reinterpret_cast<uintptr_t>(p));
}

template <int NP, int EPI, int BK, int NS>
__global__ __launch_bounds__(512) void dense_x32_kernel(const DenseX32Args a) {
  constexpr int NPL = NP == 1 ? 1 : 3, KSUB = BK / 16;
  constexpr int WQ = BK / 8, XQ = BK / 4;                          // 16-B chunks per weight / activation row
  constexpr int WPL = DX_BN * WQ, XS = DX_BM * XQ, STG = 3 * WPL + XS;   // 16-B slots
  constexpr int WBLK = WPL / 64 / 8, XBLK = XS / 64 / 8;             // DMA instructions per wave and plane
  static_assert(NS * STG * 16 <= 131072 && WBLK >= 1 && XBLK >= 1, "dense_x32 stages");
  __shared__ __attribute__((aligned(16))) uint4 L[NS * STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int wn = wave & 1, wm = wave >> 1;   // 128 weight rows x 32 activation rows per wave
  const int tile = (a.dbg & 16) ? 0 : xcd_remap(blockIdx.x, gridDim.x);   // dbg 16: every block on tile 0 (L2-resident operands)
  const int nb = tile / a.mblocks, mb = tile - nb * a.mblocks;
  const int n0 = nb * DX_BN, m0 = mb * DX_BM;
  const int nk = a.K / BK;
  const bool wactive = n0 + 128 * wn < a.N;   // wave-uniform: the wave's weight rows exist

  // DMA of k-step kt into stage st: per wave 2 x NPL weight blocks + 2 activation
  // blocks of 64 slots (rows past N / M re-read the last row; never stored)
  auto dma = [&](int kt) __attribute__((always_inline)) {
    if (a.dbg & 8) return;
    const uint4* S = L + (kt % NS) * STG;
    const int k0 = kt * BK;
#pragma unroll
    for (int p = 0; p < NPL; ++p)
#pragma unroll
      for (int j = 0; j < WBLK; ++j) {
        const int blk = WBLK * wave + j, s = 64 * blk + lane, row = s / WQ;
        const int q = dx_slot<WQ>(row, s % WQ) - WQ * row;   // the swizzle is an involution on the chunk
        const int n = min(n0 + row, a.N - 1);
        __builtin_amdgcn_global_load_lds(a.wpl + p * a.wps + (long long)n * a.K + k0 + 8 * q,
                                         dx_lds(S + p * WPL + 64 * blk), 16, 0, 0);
      }
#pragma unroll
    for (int j = 0; j < XBLK; ++j) {
      const int blk = XBLK * wave + j, s = 64 * blk + lane, row = s / XQ;
      const int c = dx_slot<XQ>(row, s % XQ) - XQ * row;
      const int m = min(m0 + row, a.M - 1);
      __builtin_amdgcn_global_load_lds(a.x + (long long)m * a.ldx + k0 + 4 * c, dx_lds(S + 3 * WPL + 64 * blk),
                                       16, 0, 0);
    }
  };

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // one k-sub (16 k) of fragments: weights 4 tiles x NPL planes, the activation
  // tile split into hi / mid / lo (each split feeds 4 x NP MFMAs)
  struct Frags {
    bf16x8 w[4][3];
    Frag3 x;
  };
  auto load = [&](int kt, int kk, Frags& f) __attribute__((always_inline)) {
    const uint4* S = L + (kt % NS) * STG;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int o = dx_slot<WQ>(128 * wn + 32 * t + l32, 2 * kk + hh);
#pragma unroll
      for (int p = 0; p < NPL; ++p) f.w[t][p] = __builtin_bit_cast(bf16x8, S[p * WPL + o]);
    }
    {
      const int row = 32 * wm + l32, c = 4 * kk + 2 * hh;
      const f32x4 x0 = __builtin_bit_cast(f32x4, S[3 * WPL + dx_slot<XQ>(row, c)]);
      const f32x4 x1 = __builtin_bit_cast(f32x4, S[3 * WPL + dx_slot<XQ>(row, c + 1)]);
      split8(x0, x1, f.x, NP == 1);
    }
  };
  auto mma = [&](const Frags& f) __attribute__((always_inline)) {
#define PPO_PL_h 0
#define PPO_PL_m 1
#define PPO_PL_l 2
#define PPO_PART(X, Y)                                 \
  _Pragma("unroll") for (int t = 0; t < 4; ++t) acc[t] = \
      __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.w[t][PPO_PL_##Y], f.x.X, acc[t], 0, 0, 0);
    PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
#undef PPO_PL_h
#undef PPO_PL_m
#undef PPO_PL_l
  };
  // interleave the next k-sub's fragment reads + split with this one's MFMAs
  auto interleave = [&]() __attribute__((always_inline)) {
    constexpr int NM = 4 * (NP == 9 ? 9 : NP == 6 ? 6 : 1);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
      if (i < 4 * NPL + 2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 LDS read
      __builtin_amdgcn_sched_group_barrier(0x002, NP == 1 ? 6 : 2, 0);   // VALU (split)
    }
  };

  // NS-stage ring, one k-sub per k-step (BK 16) or two (BK 32).  Every wave issues
  // the same DMA count per k-step (DPK), so "k-step j landed" is vmcnt <= DPK x (the
  // k-steps issued after j).  The fragments of k-sub i + 1 are read and split
  // while k-sub i's MFMAs run; a k-step's barrier comes before its first k-sub is read.
  constexpr int DPK = NPL * WBLK + XBLK;
  static_assert(DPK * 3 < 64, "vmcnt");
#define PPO_VMCNT(N) (0x0F70 | ((N) & 15) | (((N) >> 4) << 14))
  auto wait_landed = [&](int j, int issued_last) __attribute__((always_inline)) {
    const int after = issued_last - j;   // k-steps issued after j (wave-uniform)
    if (after >= 3) __builtin_amdgcn_s_waitcnt(PPO_VMCNT(DPK * 3));
    else if (after == 2) __builtin_amdgcn_s_waitcnt(PPO_VMCNT(DPK * 2));
    else if (after == 1) __builtin_amdgcn_s_waitcnt(PPO_VMCNT(DPK));
    else __builtin_amdgcn_s_waitcnt(PPO_VMCNT(0));
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };
#undef PPO_VMCNT
  int issued = -1;
  for (int j = 0; j < NS && j < nk; ++j) dma(issued = j);
  // PIPE: the next k-sub's fragments are read and split while this one's MFMAs
  // run (two fragment sets); otherwise one set, the two waves of a SIMD overlap
  // each other's split with their MFMAs
  constexpr bool PIPE = false;
  Frags fa, fb;
  if constexpr (PIPE) {
    if (nk > 0) {
      wait_landed(0, issued);
      load(0, 0, fa);
    }
  }
  const int nsub = nk * KSUB;
  for (int i = 0; i < nsub; i += 2) {
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int ii = i + h2;
      if (ii >= nsub) break;
      if constexpr (PIPE) {
        Frags& cur = h2 == 0 ? fa : fb;
        Frags& nxt = h2 == 0 ? fb : fa;
        const int nx = ii + 1;
        if (nx < nsub) {
          const int kt = nx / KSUB, kk = nx - KSUB * kt;
          if (kk == 0) {   // k-step kt opens: it must have landed; the slot of kt - 1 is free after the barrier
            wait_landed(kt, issued);
            if (kt + NS - 1 < nk && kt + NS - 1 > issued) dma(issued = kt + NS - 1);
          }
          if (wactive) {   // one basic block: the scheduler interleaves the two
            load(kt, kk, nxt);
            mma(cur);
            interleave();
          }
        } else if (wactive) {
          mma(cur);
        }
      } else {
        const int kt = ii / KSUB, kk = ii - KSUB * kt;
        if (kk == 0) {
          wait_landed(kt, issued);
          if (kt + NS - 1 < nk && kt + NS - 1 > issued) dma(issued = kt + NS - 1);
        }
        if (wactive) {
          load(kt, kk, fa);
          mma(fa);
        }
      }
    }
  }
  // Epilogue: the output tile [128 m][256 n] fp32 goes through the (free) stages in
  // chunks of CH rows (1 KB each), 16-B unit c of row m at c ^ (m & 63); every
  // wave-instruction then stores one whole 1-KB row.
  constexpr int CH = NS * STG / 64 < DX_BM ? NS * STG / 64 : DX_BM;
  static_assert(DX_BM % CH == 0 && CH % 32 == 0, "epilogue chunks");
  uint4* T = L;
#pragma unroll 1
  for (int c0 = 0; c0 < DX_BM; c0 += CH) {
    __syncthreads();   // the stages (or the previous chunk) are free
    const int m = 32 * wm + l32 - c0;
    if (wactive && m >= 0 && m < CH) {   // wave-uniform (32-row waves, chunks of 32k rows)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = (128 * wn + 32 * t + 8 * j + 4 * hh) >> 2;
          T[64 * m + (c ^ (m & 63))] = __builtin_bit_cast(
              uint4, f32x4{acc[t][4 * j], acc[t][4 * j + 1], acc[t][4 * j + 2], acc[t][4 * j + 3]});
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < CH / 8; ++i) {   // wave-instruction: one 1-KB row
      const int g = tid + 512 * i, mr = g >> 6, c = g & 63;
      const int mg = m0 + c0 + mr, n = n0 + 4 * c;
      if (mg >= a.M || n >= a.N || (a.dbg & 4)) continue;
      const f32x4 v = __builtin_bit_cast(f32x4, T[64 * mr + (c ^ (mr & 63))]);
      f32x4 y;
      if constexpr (EPI == DX_BIAS_RELU) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(a.bias + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + b[r], 0.f);
      } else {
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(a.act + (long long)mg * a.ldact + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = g4[r] > 0.f ? v[r] : 0.f;
      }
      *reinterpret_cast<f32x4*>(a.out + (long long)mg * a.ldo + n) = y;
    }
  }
}

// host side: grid = n-blocks x m-blocks (n-block-major after xcd_remap)
template <int EPI>
static int dense_x32_launch(DenseX32Args a, hipStream_t st, const char* name, int shape) {
  if (a.M <= 0 || a.N <= 0) return 0;
  PPO_REQUIRE(a.K > 0 && a.K % 32 == 0 && a.N % 4 == 0 && a.ldo % 4 == 0 && a.ldx % 4 == 0,
              "%s: K=%d must be a multiple of 32, N=%d / ldo / ldx multiples of 4", name, a.K, a.N);
  PPO_REQUIRE(((uintptr_t)a.x & 15) == 0 && ((uintptr_t)a.out & 15) == 0 && ((uintptr_t)a.wpl & 15) == 0,
              "%s: operands must be 16-B aligned", name);
  a.mblocks = (a.M + DX_BM - 1) / DX_BM;
  a.dbg = (g_stagger >> 9) & 31;
  const long long nblk = (long long)a.mblocks * ((a.N + DX_BN - 1) / DX_BN);
  PPO_REQUIRE(nblk < 0x7fffffffLL, "%s: grid too large (M=%d)", name, a.M);
  int slot;
  const bool prof = ppo_prof_begin(name, st, &slot);
  // shape 0: BK 32 x 2 stages (128 KB); 1: BK 16 x 4 stages (128 KB); 2: BK 16 x 2
  // stages (64 KB: two blocks per CU)
#define PPO_DX(NP_)                                                                                 \
  (shape == 1   ? dense_x32_kernel<NP_, EPI, 16, 4><<<(unsigned)nblk, 512, 0, st>>>(a)              \
   : shape == 2 ? dense_x32_kernel<NP_, EPI, 16, 2><<<(unsigned)nblk, 512, 0, st>>>(a)              \
                : dense_x32_kernel<NP_, EPI, 32, 2><<<(unsigned)nblk, 512, 0, st>>>(a))
  if (g_products == 9) PPO_DX(9);
  else if (g_products == 1) PPO_DX(1);
  else PPO_DX(6);
#undef PPO_DX
  if (prof) ppo_prof_end(slot, st, 2.0 * a.M * a.N * a.K);
  PPO_LAUNCH_CHECK(name);
  return 0;
}

}  // namespace
