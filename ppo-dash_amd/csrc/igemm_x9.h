// igemm_x9.h — fp32 implicit GEMM on the bf16 matrix cores, exact products.
//
// Every fp32 operand value v is split at fragment-read time into three bf16
// parts v = hi + mid + lo (exact: 3 x 8 significand bits cover fp32's 24; RNE
// at each step).  A product a·b = Σ_{p,q} a_p·b_q over the nine part pairs is
// then computed with v_mfma_f32_16x16x32_bf16, where each bf16 x bf16 product
// is exact in fp32 and the MFMA accumulates in fp32: the arithmetic of an fp32
// GEMM (exact products, fp32 accumulation; only the summation order differs,
// as between any two fp32 GEMMs), at 9 x 16 = 144 MFMA cycles per 16x16x32
// block instead of 256 on v_mfma_f32_32x32x2_f32.  An operand whose values are
// exact in bf16 (u8 pixels) uses its hi part only: 3 products.
//
// Staging is the f32 path of igemm.h (global -> registers -> LDS, double
// buffered, k-contiguous XOR-swizzled tiles), with BK = 32; loaders and
// epilogues are the same problem structs.  Row-contiguous ("non-KC") operands
// (the wgrad loaders, which load 4 rows at one k) are transposed while they are
// staged, so every LDS tile is k-contiguous.
//
// B_PLANES: the B operand (packed weights) arrives already split — three bf16
// planes written once per optimizer step by ppo_pack_weights — and is staged
// as bf16, so only the activation side is split in the k loop (by the single
// wave that owns those rows when WN = 1).
#pragma once
#include "igemm.h"

namespace {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Frag3 {
  bf16x8 h, m, l;
};

// 8 fp32 values (k-ordered) -> hi / mid / lo bf16x8 (each RNE of the residual)
__device__ __forceinline__ void split8(const f32x4& x0, const f32x4& x1, Frag3& f, bool exact) {
  const float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const bf16x2 h = __builtin_convertvector(f32x2{v[j], v[j + 1]}, bf16x2);
    f.h[j] = h[0];
    f.h[j + 1] = h[1];
    r[j] = v[j] - (float)h[0];
    r[j + 1] = v[j + 1] - (float)h[1];
  }
  if (exact) return;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const bf16x2 m = __builtin_convertvector(f32x2{r[j], r[j + 1]}, bf16x2);
    f.m[j] = m[0];
    f.m[j + 1] = m[1];
    const float r0 = r[j] - (float)m[0], r1 = r[j + 1] - (float)m[1];
    const bf16x2 l = __builtin_convertvector(f32x2{r0, r1}, bf16x2);
    f.l[j] = l[0];
    f.l[j + 1] = l[1];
  }
}

// s_waitcnt vmcnt(0) as a real S_WAITCNT (the waitcnt pass sees it, unlike inline
// asm).  Issued once after a persistent kernel's prologue loads (weights, bias):
// otherwise the pass carries those loads as pending into the image loop and its
// conservative vmcnt(N) waits there also drain the next image's prefetch.
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ f32x4 mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Part products per operand pair: NP = 9 sums all nine (exact
// products); NP = 6 (default) drops l·l, l·m and m·l, whose sum is below
// 2^-26 |a·b| — a quarter of the rounding unit of one fp32 product, so the GEMM
// keeps fp32 accuracy (the six-pass fp32 emulation, "bf16_6x").  Smallest first.
// NP = 1 is the half-precision mode (Policy.half()): bf16-rounded operands, one
// product, fp32 accumulation.
#define PPO_PRODUCTS(NP, PART)                  \
  if constexpr (NP == 9) { PART(l, l) PART(l, m) PART(m, l) } \
  if constexpr (NP >= 6) { PART(m, m) PART(l, h) PART(m, h) PART(h, l) PART(h, m) } \
  PART(h, h)

// split-product count of the launches below (ppo_tune_set("products", 1 | 6 | 9))
static int g_products = 6;
#define PPO_LAUNCH_NP(KERNEL, GRID, BLOCK, ST, ...)                   \
  do {                                                                \
    if (g_products == 9) KERNEL<9><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); \
    else if (g_products == 1) KERNEL<1><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__); \
    else KERNEL<6><<<GRID, BLOCK, 0, ST>>>(__VA_ARGS__);              \
  } while (0)

// c += Σ over the part pairs (smallest first); exact operands have hi only
template <bool AX, bool BX, int NP>
__device__ __forceinline__ f32x4 mma9(const Frag3& a, const Frag3& b, f32x4 c) {
  if constexpr (NP == 1) return mma(a.h, b.h, c);   // half-precision mode
  if constexpr (!AX && !BX) {
    if constexpr (NP == 9) {
      c = mma(a.l, b.l, c);
      c = mma(a.l, b.m, c);
      c = mma(a.m, b.l, c);
    }
    c = mma(a.m, b.m, c);
  }
  if constexpr (!AX) {
    c = mma(a.l, b.h, c);
    c = mma(a.m, b.h, c);
  }
  if constexpr (!BX) {
    c = mma(a.h, b.l, c);
    c = mma(a.h, b.m, c);
  }
  return mma(a.h, b.h, c);
}

// BM x BN block, WM x WN waves of (BM/WM) x (BN/WN), 16x16 MFMA tiles, BK 32.
// AX / BX: operand values are exact in bf16 (u8 data).
template <int BM_, int BN_, int WM_, int WN_, bool AKC, bool BKC, bool BIASA = false, bool AX_ = false,
          bool BX_ = false, bool BP_ = false>
struct CfgX {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NT = 64 * WM_ * WN_, BK = 32;
  static constexpr bool A_KC = AKC, B_KC = BKC, BIAS_FROM_A = BIASA, TILE_EPI = false, B_TILE = false;
  static constexpr bool A_EXACT = AX_, B_EXACT = BX_, B_PLANES = BP_, SPLIT_STAGE = false, VEC_STORE = false;
  int vec = 0;
  struct ACtx { const float* p; int a; int b; bool ok; };
  struct BCtx { const float* p; int a; bool ok; };
  // B_PLANES: plane p of B[n][k] at bpl[p * bps + n * bld + k] (bf16 bits), n < bnr, k < bld
  const uint16_t* bpl = nullptr;
  long long bps = 0;
  int bld = 0, bnr = 0;
  // tile order (see igemm_x9_kernel): 1 = (z, m, n) n fastest per XCD, for an A operand
  // larger than the Infinity Cache shared by N / BN tiles (fc forward); 0 = m fastest
  // (each XCD sweeps its m range at one n: B tile L2-resident, A from the Infinity Cache)
  int n_fast = 0;
};

// LDS swizzles for the 16x16x32 fragment reads.  ds_read_b128 serves a wave in
// four 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
// {36-43,48-51,60-63} (MI355X_MICROARCH.md §LDS); lane l reads row l & 15,
// chunk(s) of lane group l >> 4.  A group is conflict-free when its 16 reads hit
// 16 distinct 16-B slots of the 256-B bank row:
//  * f32 tile, 128-B rows (8 chunks), chunks 2g and 2g+1: chunk q of row r at
//    q ^ H8[(r >> 1) & 7] with H8 = {0,1,4,5,6,7,2,3} (rows {0-3,12-15} and
//    {4-11} must draw disjoint XOR sets that are each closed under ^2);
//  * bf16 plane, 64-B rows (4 chunks), chunk g: chunk q at q ^ H4[(r >> 2) & 3],
//    H4 = {0,2,3,1}.
// The staging ds_write_b128 (8 contiguous lanes, 128-B bank rows) of one row's
// chunks is a permutation of one row: conflict-free for both.
__device__ __forceinline__ int x9_off(int row, int k) {   // f32 element offset, k multiple of 4
  constexpr unsigned H8 = 0x32765410u;   // nibbles: H8[i] = (H8 >> 4i) & 15
  return row * 32 + 4 * ((k >> 2) ^ ((H8 >> (4 * ((row >> 1) & 7))) & 7));
}
// pl_off also swaps rows 2j, 2j + 1 in every second group of 16 rows (row bit 0 ^=
// bit 4): the split-at-staging kernel's non-KC units write rows 4t + q of 8
// consecutive t from 8 lanes at one chunk, which without it all sit in the same
// 64-B quarter of the 256-B bank row (2-way conflicts: 31 % of the fc weight
// gradient's LDS cycles, profiles/r05_s_fc_sq.json); with it those 8 writes, the 2-row
// x 4-chunk KC writes and the ds_read_b128 fragment groups are all conflict-free
// (exhaustive check over the tile, tools/swizzle_check.py).
__device__ __forceinline__ int pl_off(int row, int q) {   // bf16 element offset
  constexpr unsigned H4 = 0x1320u;
  return (row ^ ((row >> 4) & 1)) * 32 + 8 * (q ^ ((H4 >> (4 * ((row >> 2) & 3))) & 3));
}

// Block -> (m0, n0, z) tile.  n_fast 0: m = xcd_remap(blockIdx.x) (each XCD a
// contiguous m range), n = blockIdx.y, z = blockIdx.z — the dispatcher walks all m
// at one n before the next n, so the B tile stays L2-resident and A (if it fits the
// 256 MB Infinity Cache) is re-read from there.  n_fast 1: (z, m, n) with n fastest,
// dealt out by xcd_remap of the linear block id so the N / BN tiles that share an
// A row tile (and the tiles of one split-K slice, which share its rows) run at the
// same time on one XCD and read the common operand from that XCD's L2 — for an A
// operand larger than the Infinity Cache (fc forward: 411 MB, re-streamed from HBM
// by each of the 4 tile columns with n_fast 0: 0.625 -> 0.56 ms).
__device__ __forceinline__ void tile_of(int n_fast, int BM, int BN, int& m0, int& n0, int& z) {
  if (!n_fast) {
    m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
    n0 = blockIdx.y * BN;
    z = blockIdx.z;
    return;
  }
  const int gx = (int)gridDim.x, gy = (int)gridDim.y, mn = gx * gy;
  const int lin = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
  const int t = xcd_remap(lin, mn * (int)gridDim.z);
  z = t / mn;
  const int r = t - z * mn, mt = r / gy;
  m0 = mt * BM;
  n0 = (r - mt * gy) * BN;
}

// Vector epilogue of a wave's TM x TN 16x16 tiles: each tile goes through the
// wave's own 16 x 17-float slice of the (free) LDS so that every lane stores four
// consecutive columns of one row (one 16-B store, and 16-B operand loads in the
// problem's store4) instead of one column of four rows (4-B accesses in 64-B runs):
// fc forward 0.565 -> 0.542, fc dgrad 0.723 -> 0.680 ms at the c3 minibatch.
template <class P, int TM, int TN>
__device__ __forceinline__ void vec_epilogue(const P& p, float* smem, const f32x4 (&acc)[TM][TN], int wave, int lane,
                                             int mb, int nb, int z) {
  float* T = smem + wave * (16 * 17);
  const int fr = lane & 15, fg = lane >> 4, tr = lane >> 2, tc = 4 * (lane & 3);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(4 * fg + r) * 17 + fr] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
      const f32x4 v = {T[tr * 17 + tc], T[tr * 17 + tc + 1], T[tr * 17 + tc + 2], T[tr * 17 + tc + 3]};
      __builtin_amdgcn_wave_barrier();
      p.store4(mb + i * 16 + tr, nb + j * 16 + tc, z, v);
    }
}

// one 16-B chunk of B plane pl, row n, from k: a branch-free buffer load (a row past
// bnr or k past bld is sent out of the 3-plane resource's range and reads 0);
// launch_x9 checks 6·bps < 2^31
template <class P>
__device__ __forceinline__ uint4 bpl_load(const P& p, int n, int pl, int kk) {
  const uint32_t off = (n < p.bnr && kk < p.bld)
                           ? 2u * ((uint32_t)pl * (uint32_t)p.bps + (uint32_t)n * (uint32_t)p.bld + (uint32_t)kk)
                           : 0x80000000u;
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(p.bpl, 6u * (uint32_t)p.bps), off, 0, 0));
}

template <class P, int NP>
__global__ __launch_bounds__(P::NT) void igemm_x9_kernel(const P p) {
  constexpr int BM = P::BM, BN = P::BN, NT = P::NT, WM = P::WM, WN = P::WN, BK = 32;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(TM * 16 * WM == BM && TN * 16 * WN == BN && WM * WN * 64 == NT, "tile config");
  static_assert(BM % 4 == 0 && BN % 4 == 0, "rows");
  constexpr bool BPL = P::B_PLANES;
  constexpr int SA = BM * BK, SB = BPL ? BN * BK * 3 / 2 : BN * BK, STAGE = SA + SB;   // floats
  // staging units: KC operand -> one 4-k chunk of one row; non-KC operand -> a
  // 4-row x 8-k block (8 row-vector loads, transposed into 2 chunks per row)
  constexpr int UA = P::A_KC ? BM * BK / 4 : (BM / 4) * (BK / 8);
  constexpr int UB = BPL ? BN * 12 : P::B_KC ? BN * BK / 4 : (BN / 4) * (BK / 8);
  constexpr int NUA = (UA + NT - 1) / NT, NUB = (UB + NT - 1) / NT;
  constexpr int LA = P::A_KC ? 1 : 8, LB = P::B_KC ? 1 : 8;   // loads per unit
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int m0, n0, z;
  tile_of(p.n_fast, BM, BN, m0, n0, z);
  int kbeg, kend;
  p.k_range(z, kbeg, kend);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  typename P::ACtx actx[NUA];
  typename P::BCtx bctx[NUB];
  int ak[NUA], arow[NUA], bk[NUB], brow[NUB];
  bool aon[NUA], bon[NUB];
#pragma unroll
  for (int i = 0; i < NUA; ++i) {
    const int u = tid + i * NT;
    aon[i] = (i + 1) * NT <= UA || u < UA;   // a full row of units: known true, no exec mask
    if constexpr (P::A_KC) {
      arow[i] = u / (BK / 4);
      ak[i] = 4 * (u % (BK / 4));
    } else {
      arow[i] = 4 * (u % (BM / 4));
      ak[i] = 8 * (u / (BM / 4));
    }
    actx[i] = p.a_ctx(m0 + arow[i], z);
  }
#pragma unroll
  for (int i = 0; i < NUB; ++i) {
    const int u = tid + i * NT;
    bon[i] = (i + 1) * NT <= UB || u < UB;
    if constexpr (BPL) {   // brow = plane row, bk = plane * 4 + 16-B chunk
      brow[i] = (u % (BN * 4)) / 4;
      bk[i] = (u / (BN * 4)) * 4 + u % 4;
      bctx[i] = typename P::BCtx{};
      continue;
    }
    if constexpr (P::B_KC) {
      brow[i] = u / (BK / 4);
      bk[i] = 4 * (u % (BK / 4));
    } else {
      brow[i] = 4 * (u % (BN / 4));
      bk[i] = 8 * (u / (BN / 4));
    }
    bctx[i] = p.b_ctx(n0 + brow[i], z);
  }

  using ARaw = decltype(p.a_load(actx[0], 0));
  auto bload = [&](int i, int k) {
    if constexpr (BPL) {   // k = k0 + bk[i]: plane bk >> 2, chunk bk & 3
      const int n = n0 + brow[i], pl = (k - (k & ~(BK - 1))) >> 2, kk = (k & ~(BK - 1)) + 8 * (k & 3);
      return bpl_load(p, n, pl, kk);
    } else if constexpr (P::B_TILE) {
      return p.b_load_t(bctx[i], p.tile(k & ~(BK - 1)), k);
    } else {
      return p.b_load(bctx[i], k);
    }
  };
  using BRaw = decltype(bload(0, 0));
  ARaw ra[NUA][LA];
  BRaw rb[NUB][BPL ? 1 : LB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NUA; ++i)
#pragma unroll
      for (int j = 0; j < LA; ++j) ra[i][j] = aon[i] ? p.a_load(actx[i], k0 + ak[i] + j) : ARaw{};
#pragma unroll
    for (int i = 0; i < NUB; ++i) {
      if constexpr (BPL) {
        rb[i][0] = bon[i] ? bload(i, k0 + bk[i]) : BRaw{};
      } else {
#pragma unroll
        for (int j = 0; j < LB; ++j) rb[i][j] = bon[i] ? bload(i, k0 + bk[i] + j) : BRaw{};
      }
    }
  };
  // non-KC unit: v[j] = rows r..r+3 at k+j  ->  row r+q gets k..k+3 and k+4..k+7
  auto put_t = [&](float* S, int row, int k, const f32x4 (&v)[8]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *reinterpret_cast<f32x4*>(S + x9_off(row + q, k)) = f32x4{v[0][q], v[1][q], v[2][q], v[3][q]};
      *reinterpret_cast<f32x4*>(S + x9_off(row + q, k + 4)) = f32x4{v[4][q], v[5][q], v[6][q], v[7][q]};
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * STAGE;
    float* Bs = As + SA;
#pragma unroll
    for (int i = 0; i < NUA; ++i) {
      if (!aon[i]) continue;
      if constexpr (P::A_KC) {
        *reinterpret_cast<f32x4*>(As + x9_off(arow[i], ak[i])) = to_f32x4(ra[i][0]);
      } else {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = to_f32x4(ra[i][j]);
        put_t(As, arow[i], ak[i], v);
      }
    }
#pragma unroll
    for (int i = 0; i < NUB; ++i) {
      if (!bon[i]) continue;
      if constexpr (BPL) {
        uint16_t* Bp = reinterpret_cast<uint16_t*>(Bs) + (bk[i] >> 2) * (BN * 32);
        *reinterpret_cast<uint4*>(Bp + pl_off(brow[i], bk[i] & 3)) = rb[i][0];
      } else if constexpr (P::B_KC) {
        *reinterpret_cast<f32x4*>(Bs + x9_off(brow[i], bk[i])) = to_f32x4(rb[i][0]);
      } else {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = to_f32x4(rb[i][j]);
        put_t(Bs, brow[i], bk[i], v);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  float bias_acc = 0.f;

  const int fr = lane & 15, fg = lane >> 4;
  auto frag = [&](const float* S, int row, Frag3& f, bool exact) {
    const f32x4 x0 = *reinterpret_cast<const f32x4*>(S + x9_off(row, 8 * fg));
    const f32x4 x1 = *reinterpret_cast<const f32x4*>(S + x9_off(row, 8 * fg + 4));
    split8(x0, x1, f, exact);
  };

  if (nk > 0) {
    gload(kbeg);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kbeg + (kt + 1) * BK);
    const float* As = smem + buf * STAGE;
    const float* Bs = As + SA;
    if constexpr (P::BIAS_FROM_A) {   // db partial: thread sums BK/G k of one A row
      static_assert(NT % BM == 0 && BK % (NT / BM) == 0, "bias partials");
      constexpr int G = NT / BM;
      if (n0 == 0) {
        const int row = tid % BM;
#pragma unroll
        for (int k = (tid / BM) * 4; k < BK; k += 4 * G) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(As + x9_off(row, k));
          bias_acc += (v[0] + v[1]) + (v[2] + v[3]);
        }
      }
    }
    if constexpr (BPL) {
      const uint16_t* Bp = reinterpret_cast<const uint16_t*>(Bs);
      Frag3 fa[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) frag(As, (wm * TM + i) * 16 + fr, fa[i], P::A_EXACT);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = (wn * TN + j) * 16 + fr, o = pl_off(row, fg);
        Frag3 fb;
        fb.h = *reinterpret_cast<const bf16x8*>(Bp + o);
        fb.m = *reinterpret_cast<const bf16x8*>(Bp + BN * 32 + o);
        fb.l = *reinterpret_cast<const bf16x8*>(Bp + 2 * BN * 32 + o);
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mma9<P::A_EXACT, false, NP>(fa[i], fb, acc[i][j]);
      }
    } else {
      Frag3 fb[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) frag(Bs, (wn * TN + j) * 16 + fr, fb[j], P::B_EXACT);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        Frag3 fa;
        frag(As, (wm * TM + i) * 16 + fr, fa, P::A_EXACT);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mma9<P::A_EXACT, P::B_EXACT, NP>(fa, fb[j], acc[i][j]);
      }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  bool vec_done = false;
  if constexpr (P::VEC_STORE) {
    if (p.vec) {   // the main loop ended on a barrier: the LDS is free
      vec_epilogue<P, TM, TN>(p, smem, acc, wave, lane, m0 + wm * TM * 16, n0 + wn * TN * 16, z);
      vec_done = true;
    }
  }
  if (!vec_done) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          p.store(m0 + (wm * TM + i) * 16 + 4 * fg + r, n0 + (wn * TN + j) * 16 + fr, z, acc[i][j][r]);
  }
  if constexpr (P::BIAS_FROM_A) {
    if (n0 == 0) {   // fixed-order combine of the G partials of each row
      __syncthreads();   // the vector epilogue's LDS slices are read
      constexpr int G = NT / BM;
      smem[tid] = bias_acc;   // the main loop ended on a barrier
      __syncthreads();
      if (tid < BM) {
        float t = smem[tid];
#pragma unroll
        for (int g = 1; g < G; ++g) t += smem[g * BM + tid];
        p.store_bias(m0 + tid, z, t);
      }
    }
  }
}

// Split-at-staging form (igemm_x9s_kernel, configs CfgS): the fp32 operands are
// split ONCE per block, while they are staged, into three bf16 planes in LDS
// (64-B rows, pl_off swizzle), and the k loop reads plain bf16 fragments — no
// split VALU in the k loop, and no operand split again by every wave that reads
// it (igemm_x9_kernel splits each fragment in each wave: with WM x WN waves a B
// row is split WM times; the fc weight gradient's 4 x 2 waves split B 4x and A 2x
// per k-step, which made it VALU-issue-bound, 0.32 of the MFMA roofline).
//   KC operand (row-contiguous k): unit = one row x 8 k (two 16-B loads);
//   non-KC operand (wgrad: k = sample row): unit = 4 rows x 8 k (eight 16-B loads
//   of 4 consecutive rows at one k), transposed while split.
// A and B units are dealt to threads from opposite ends so that the threads the A
// units leave idle take the B units.  BIAS_FROM_A (wgrad bias partial): each
// thread sums its A unit's 4 rows over its 8 k per step; the four k-groups of a row
// are combined in a fixed order at the end.
template <int BM_, int BN_, int WM_, int WN_, bool AKC, bool BKC, bool BIASA = false, bool BP_ = false>
struct CfgS : CfgX<BM_, BN_, WM_, WN_, AKC, BKC, BIASA, false, false, BP_> {
  static constexpr bool SPLIT_STAGE = true;
};

template <class P, int NP>
__global__ __launch_bounds__(P::NT) void igemm_x9s_kernel(const P p) {
  constexpr int BM = P::BM, BN = P::BN, NT = P::NT, WM = P::WM, WN = P::WN, BK = 32;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(TM * 16 * WM == BM && TN * 16 * WN == BN && WM * WN * 64 == NT, "tile config");
  static_assert(!P::A_EXACT && !P::B_EXACT, "split staging: fp32 operands");
  constexpr bool BPL = P::B_PLANES, AKC = P::A_KC, BKC = P::B_KC;
  constexpr int NPL = NP == 1 ? 1 : 3;                      // planes staged
  constexpr int PA = BM * BK, PB = BN * BK;                 // bf16 elements per plane
  constexpr int STAGE = NPL * PA + (BPL ? 3 : NPL) * PB;    // bf16 elements per stage
  constexpr int UA = AKC ? BM * 4 : (BM / 4) * 4;
  constexpr int UB = BPL ? BN * 12 : BKC ? BN * 4 : (BN / 4) * 4;
  constexpr int NUA = (UA + NT - 1) / NT, NUB = (UB + NT - 1) / NT;
  constexpr int LA = AKC ? 2 : 8, LB = BPL ? 1 : BKC ? 2 : 8;
  constexpr int BOFF = (NT - UA % NT) % NT;                 // B units start where the A units end
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * STAGE];
  static_assert(!P::BIAS_FROM_A || (!AKC && UA <= NT && BM * 8 <= 2 * STAGE), "bias partials: wgrad layout");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int m0, n0, z;
  tile_of(p.n_fast, BM, BN, m0, n0, z);
  int kbeg, kend;
  p.k_range(z, kbeg, kend);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  typename P::ACtx actx[NUA];
  typename P::BCtx bctx[NUB];
  int ak[NUA], arow[NUA], bk[NUB], brow[NUB];
  bool aon[NUA], bon[NUB];
#pragma unroll
  for (int i = 0; i < NUA; ++i) {
    const int u = tid + i * NT;
    aon[i] = (i + 1) * NT <= UA || u < UA;   // a full row of units: known true, no exec mask
    if constexpr (AKC) {
      arow[i] = u >> 2;
      ak[i] = 8 * (u & 3);
    } else {
      arow[i] = 4 * (u % (BM / 4));
      ak[i] = 8 * (u / (BM / 4));
    }
    actx[i] = p.a_ctx(m0 + (aon[i] ? arow[i] : 0), z);
  }
#pragma unroll
  for (int i = 0; i < NUB; ++i) {
    const int u = (tid + BOFF) % NT + i * NT;
    bon[i] = (i + 1) * NT <= UB || u < UB;
    if constexpr (BPL) {   // brow = plane row, bk = plane * 4 + 16-B chunk
      brow[i] = (u % (BN * 4)) / 4;
      bk[i] = (u / (BN * 4)) * 4 + u % 4;
      bctx[i] = typename P::BCtx{};
      continue;
    }
    if constexpr (BKC) {
      brow[i] = u >> 2;
      bk[i] = 8 * (u & 3);
    } else {
      brow[i] = 4 * (u % (BN / 4));
      bk[i] = 8 * (u / (BN / 4));
    }
    bctx[i] = p.b_ctx(n0 + (bon[i] ? brow[i] : 0), z);
  }

  using ARaw = decltype(p.a_load(actx[0], 0));
  auto bload = [&](int i, int k) {
    if constexpr (BPL) {   // k = k0 + bk[i]: plane bk >> 2, chunk bk & 3
      const int n = n0 + brow[i], pl = (k - (k & ~(BK - 1))) >> 2, kk = (k & ~(BK - 1)) + 8 * (k & 3);
      return bpl_load(p, n, pl, kk);
    } else {
      return p.b_load(bctx[i], k);
    }
  };
  using BRaw = decltype(bload(0, 0));
  ARaw ra[NUA][LA];
  BRaw rb[NUB][LB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NUA; ++i)
#pragma unroll
      for (int j = 0; j < LA; ++j) ra[i][j] = aon[i] ? p.a_load(actx[i], k0 + ak[i] + (AKC ? 4 * j : j)) : ARaw{};
#pragma unroll
    for (int i = 0; i < NUB; ++i)
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        if constexpr (BPL) rb[i][j] = bon[i] ? bload(i, k0 + bk[i]) : BRaw{};
        else rb[i][j] = bon[i] ? bload(i, k0 + bk[i] + (BKC ? 4 * j : j)) : BRaw{};
      }
  };
  float bias_acc[4] = {0.f, 0.f, 0.f, 0.f};   // BIAS_FROM_A: rows arow[0] + q, this thread's k-group
  // 8 fp32 (k-ordered) -> the planes of one 16-B chunk of row `row`
  auto put8 = [&](uint16_t* S, int pstride, int row, int q, const f32x4& x0, const f32x4& x1) {
    Frag3 f;
    split8(x0, x1, f, NP == 1);
    const int o = pl_off(row, q);
    *reinterpret_cast<bf16x8*>(S + o) = f.h;
    if constexpr (NPL == 3) {
      *reinterpret_cast<bf16x8*>(S + pstride + o) = f.m;
      *reinterpret_cast<bf16x8*>(S + 2 * pstride + o) = f.l;
    }
  };
  auto sstore = [&](int buf, bool bias_on) {
    uint16_t* As = smem + buf * STAGE;
    uint16_t* Bs = As + NPL * PA;
#pragma unroll
    for (int i = 0; i < NUA; ++i) {
      if (!aon[i]) continue;
      if constexpr (AKC) {
        put8(As, PA, arow[i], ak[i] >> 3, to_f32x4(ra[i][0]), to_f32x4(ra[i][1]));
      } else {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = to_f32x4(ra[i][j]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 x0 = {v[0][q], v[1][q], v[2][q], v[3][q]}, x1 = {v[4][q], v[5][q], v[6][q], v[7][q]};
          put8(As, PA, arow[i] + q, ak[i] >> 3, x0, x1);
          if constexpr (P::BIAS_FROM_A)
            if (bias_on) bias_acc[q] += ((x0[0] + x0[1]) + (x0[2] + x0[3])) + ((x1[0] + x1[1]) + (x1[2] + x1[3]));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NUB; ++i) {
      if (!bon[i]) continue;
      if constexpr (BPL) {
        *reinterpret_cast<uint4*>(Bs + (bk[i] >> 2) * PB + pl_off(brow[i], bk[i] & 3)) = rb[i][0];
      } else if constexpr (BKC) {
        put8(Bs, PB, brow[i], bk[i] >> 3, to_f32x4(rb[i][0]), to_f32x4(rb[i][1]));
      } else {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = to_f32x4(rb[i][j]);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          put8(Bs, PB, brow[i] + q, bk[i] >> 3, f32x4{v[0][q], v[1][q], v[2][q], v[3][q]},
               f32x4{v[4][q], v[5][q], v[6][q], v[7][q]});
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();

  const int fr = lane & 15, fg = lane >> 4;
  const bool bias_on = P::BIAS_FROM_A && n0 == 0;
  if (nk > 0) {
    gload(kbeg);
    sstore(0, bias_on);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kbeg + (kt + 1) * BK);
    const uint16_t* As = smem + buf * STAGE;
    const uint16_t* Bs = As + NPL * PA;
    Frag3 fb[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = pl_off((wn * TN + j) * 16 + fr, fg);
      fb[j].h = *reinterpret_cast<const bf16x8*>(Bs + o);
      if constexpr (NPL == 3) {
        fb[j].m = *reinterpret_cast<const bf16x8*>(Bs + PB + o);
        fb[j].l = *reinterpret_cast<const bf16x8*>(Bs + 2 * PB + o);
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int o = pl_off((wm * TM + i) * 16 + fr, fg);
      Frag3 fa;
      fa.h = *reinterpret_cast<const bf16x8*>(As + o);
      if constexpr (NPL == 3) {
        fa.m = *reinterpret_cast<const bf16x8*>(As + PA + o);
        fa.l = *reinterpret_cast<const bf16x8*>(As + 2 * PA + o);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mma9<false, false, NP>(fa, fb[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1, bias_on);
    __syncthreads();
  }

  bool vec_done = false;
  if constexpr (P::VEC_STORE) {
    if (p.vec) {   // the main loop ended on a barrier: the LDS is free
      vec_epilogue<P, TM, TN>(p, reinterpret_cast<float*>(smem), acc, wave, lane, m0 + wm * TM * 16, n0 + wn * TN * 16,
                              z);
      vec_done = true;
    }
  }
  if (!vec_done) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          p.store(m0 + (wm * TM + i) * 16 + 4 * fg + r, n0 + (wn * TN + j) * 16 + fr, z, acc[i][j][r]);
  }
  if constexpr (P::BIAS_FROM_A) {
    if (bias_on) {   // row r: its four k-groups' partials, fixed order (k0 + k1) + (k2 + k3)
      __syncthreads();   // the vector epilogue's LDS slices are read
      float* red = reinterpret_cast<float*>(smem);
      if (aon[0])
#pragma unroll
        for (int q = 0; q < 4; ++q) red[(ak[0] >> 3) * BM + arow[0] + q] = bias_acc[q];
      __syncthreads();
      if (tid < BM) p.store_bias(m0 + tid, z, (red[tid] + red[BM + tid]) + (red[2 * BM + tid] + red[3 * BM + tid]));
    }
  }
}

template <class P>
int launch_x9(const P& p, long long M, int N, int Z, hipStream_t st, const char* name, double flops) {
  if (M <= 0 || N <= 0 || Z <= 0) return 0;
  const long long gx = (M + P::BM - 1) / P::BM;
  if (gx > 0x7fffffffLL) {
    ppo_set_error("%s: grid too large (M=%lld)", name, M);
    return PPO_ESHAPE;
  }
  if constexpr (P::B_PLANES) {
    if (6LL * p.bps >= 0x80000000LL) {   // bpl_load's 32-bit offsets
      ppo_set_error("%s: B planes too large (%lld elements)", name, p.bps);
      return PPO_ESHAPE;
    }
  }
  dim3 grid((unsigned)gx, (unsigned)((N + P::BN - 1) / P::BN), (unsigned)Z);
  int slot;
  const bool prof = ppo_prof_begin(name, st, &slot);
  if constexpr (P::SPLIT_STAGE) {
    if (g_products == 9) igemm_x9s_kernel<P, 9><<<grid, P::NT, 0, st>>>(p);
    else if (g_products == 1) igemm_x9s_kernel<P, 1><<<grid, P::NT, 0, st>>>(p);
    else igemm_x9s_kernel<P, 6><<<grid, P::NT, 0, st>>>(p);
  } else {
    if (g_products == 9) igemm_x9_kernel<P, 9><<<grid, P::NT, 0, st>>>(p);
    else if (g_products == 1) igemm_x9_kernel<P, 1><<<grid, P::NT, 0, st>>>(p);
    else igemm_x9_kernel<P, 6><<<grid, P::NT, 0, st>>>(p);
  }
  if (prof) ppo_prof_end(slot, st, flops);
  PPO_LAUNCH_CHECK(name);
  return 0;
}

}  // namespace
