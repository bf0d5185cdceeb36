// igemm.h — the fp32-MFMA implicit-GEMM core shared by the CNN trunk
// (gemm.hip) and the GRU (gru.hip).  See gemm.hip's header for the design.
#pragma once
#include <string.h>

#include "common.h"

namespace {

constexpr int BK16 = 16;  // default k-tile depth (wgrad chunks are multiples of it)

// k-contiguous tiles: rows of BK floats (CPR = BK/4 16-B chunks), chunk q of
// row r stored at chunk q ^ f(r), f(r) = (r / (16/CPR)) mod CPR.  A wave's
// fragment read (32 rows, one chunk each) then hits 16 distinct 16-B slots in
// every ds_read_b128 lane group, and the staging ds_write_b128 of whole rows is
// contiguous — both conflict-free (PMC: SQ_LDS_BANK_CONFLICT, the +4 padding
// this replaces cost 37 % of LDS cycles in the staging writes).
template <int ROWS, bool KC, int BK>
struct Tile {
  static constexpr int LD = BK;
  static constexpr int SIZE = KC ? ROWS * LD : BK * ROWS;
  static constexpr int NV4 = ROWS * BK / 4;
};

template <int BK>
__device__ __forceinline__ int kc_off(int row, int k) {  // k multiple of 4
  constexpr int CPR = BK / 4;
  const int q = (k >> 2) ^ ((row / (16 / CPR)) & (CPR - 1));
  return row * BK + 4 * q;
}

template <int ROWS, bool KC, int BK>
__device__ __forceinline__ f32x4 frag(const float* S, int row, int kb) {
  if constexpr (KC) {
    return *reinterpret_cast<const f32x4*>(S + kc_off<BK>(row, kb));
  } else {
    f32x4 r;
    r[0] = S[(kb + 0) * ROWS + row];
    r[1] = S[(kb + 1) * ROWS + row];
    r[2] = S[(kb + 2) * ROWS + row];
    r[3] = S[(kb + 3) * ROWS + row];
    return r;
  }
}

// Bijective XCD-aware remap (guide §5.5 T1): blocks that share an XCD
// (b ≡ b' mod 8) get consecutive tiles, so neighbouring im2col windows and
// weight tiles are served from that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nb) {
  const int xcd = bid & 7, q = nb >> 3, r = nb & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// Operand loaders return their raw global data (f32x4, or uint32_t = 4 u8
// pixels); the conversion to the f32 MFMA operand runs at the LDS store, after
// the current tile's MFMAs, so a tile's global loads stay in flight across the
// whole compute phase instead of stalling the wave right after issue.
__device__ __forceinline__ f32x4 to_f32x4(const f32x4& v) { return v; }
__device__ __forceinline__ f32x4 to_f32x4(uint32_t u) {
  return f32x4{(float)(u & 255u), (float)((u >> 8) & 255u), (float)((u >> 16) & 255u), (float)(u >> 24)};
}

// ---------------------------------------------------------------------------
// Core: C[m][n] = Σ_k A[m][k] B[n][k]; problem P supplies loaders + epilogue.
// ---------------------------------------------------------------------------
template <class P>
__global__ __launch_bounds__(P::NT) void igemm_kernel(const P p) {
  constexpr int BM = P::BM, BN = P::BN, NT = P::NT, WM = P::WM, WN = P::WN, BK = P::BK;
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
  static_assert(TM * 32 * WM == BM && TN * 32 * WN == BN && WM * WN * 64 == NT, "tile config");
  static_assert(BK == 16 || BK == 32, "k-tile");
  using TA = Tile<BM, P::A_KC, BK>;
  using TB = Tile<BN, P::B_KC, BK>;
  constexpr int NVA = (TA::NV4 + NT - 1) / NT, NVB = (TB::NV4 + NT - 1) / NT;
  constexpr int STAGE = TA::SIZE + TB::SIZE;
#ifndef PPO_GEMM_STAGES
#define PPO_GEMM_STAGES 2
#endif
  // 2: double-buffered LDS, fragments read at the start of each 8-deep k group.
  // 3: triple-buffered LDS; a wave reads the next k group's fragments (across
  //    the k-tile boundary too: tile t+1 is already staged) while its MFMAs on
  //    the current group run, so LDS latency never sits in front of an MFMA.
  constexpr int NS = PPO_GEMM_STAGES;
  static_assert(NS == 2 || NS == 3, "stages");
  __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int n0 = blockIdx.y * BN;
  const int z = blockIdx.z;
  int kbeg, kend;
  p.k_range(z, kbeg, kend);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  typename P::ACtx actx[NVA];
  typename P::BCtx bctx[NVB];
  int ak[NVA], aoff[NVA], bk[NVB], boff[NVB];
  bool aon[NVA], bon[NVB];
#pragma unroll
  for (int i = 0; i < NVA; ++i) {
    const int f = tid + i * NT;
    aon[i] = f < TA::NV4;
    if constexpr (P::A_KC) {
      const int row = f / (BK / 4), kq = f % (BK / 4);
      actx[i] = p.a_ctx(m0 + row, z);
      ak[i] = 4 * kq;
      aoff[i] = kc_off<BK>(row, 4 * kq);
    } else {
      const int k = f / (BM / 4), rq = f % (BM / 4);
      actx[i] = p.a_ctx(m0 + 4 * rq, z);
      ak[i] = k;
      aoff[i] = k * BM + 4 * rq;
    }
  }
#pragma unroll
  for (int i = 0; i < NVB; ++i) {
    const int f = tid + i * NT;
    bon[i] = f < TB::NV4;
    if constexpr (P::B_KC) {
      const int row = f / (BK / 4), kq = f % (BK / 4);
      bctx[i] = p.b_ctx(n0 + row, z);
      bk[i] = 4 * kq;
      boff[i] = kc_off<BK>(row, 4 * kq);
    } else {
      const int k = f / (BN / 4), rq = f % (BN / 4);
      bctx[i] = p.b_ctx(n0 + 4 * rq, z);
      bk[i] = k;
      boff[i] = k * BN + 4 * rq;
    }
  }

  using ARaw = decltype(p.a_load(actx[0], 0));
  ARaw ra[NVA];
  // B loaders may take a per-k-tile context computed once from the (block-
  // uniform) tile start, e.g. the image a 16-row wgrad tile lies in.
  auto bload = [&](int i, int k0) {
    if constexpr (P::B_TILE) return p.b_load_t(bctx[i], p.tile(k0), k0 + bk[i]);
    else return p.b_load(bctx[i], k0 + bk[i]);
  };
  using BRaw = decltype(bload(0, 0));
  BRaw rb[NVB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NVA; ++i) ra[i] = aon[i] ? p.a_load(actx[i], k0 + ak[i]) : ARaw{};
#pragma unroll
    for (int i = 0; i < NVB; ++i) rb[i] = bon[i] ? bload(i, k0) : BRaw{};
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * STAGE;
    float* Bs = As + TA::SIZE;
#pragma unroll
    for (int i = 0; i < NVA; ++i)
      if (aon[i]) *reinterpret_cast<f32x4*>(As + aoff[i]) = to_f32x4(ra[i]);
#pragma unroll
    for (int i = 0; i < NVB; ++i)
      if (bon[i]) *reinterpret_cast<f32x4*>(Bs + boff[i]) = to_f32x4(rb[i]);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float bias_acc = 0.f;

  const int frow = lane & 31, fk = 4 * (lane >> 5);
  auto bias_part = [&](const float* As) {
    if constexpr (P::BIAS_FROM_A) {
      // db partial: every thread sums BK/G rows of one A-tile column
      static_assert(!P::A_KC && NT % BM == 0 && BK % (NT / BM) == 0, "bias partials");
      constexpr int G = NT / BM;
      if (blockIdx.y == 0) {
#pragma unroll
        for (int k = tid / BM; k < BK; k += G) bias_acc += As[k * BM + tid % BM];
      }
    }
  };
  auto read_frags = [&](const float* As, int kb, f32x4 (&af)[TM], f32x4 (&bf)[TN]) {
    const float* Bs = As + TA::SIZE;
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = frag<BM, P::A_KC, BK>(As, (wm * TM + i) * 32 + frow, kb + fk);
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = frag<BN, P::B_KC, BK>(Bs, (wn * TN + j) * 32 + frow, kb + fk);
  };
  auto mfma_group = [&](const f32x4 (&af)[TM], const f32x4 (&bf)[TN]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
  };

  if constexpr (NS == 2) {
    if (nk > 0) {
      gload(kbeg);
      sstore(0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) gload(kbeg + (kt + 1) * BK);
      const float* As = smem + buf * STAGE;
      bias_part(As);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 8) {
        f32x4 af[TM], bf[TN];
        read_frags(As, kk, af, bf);
        mfma_group(af, bf);
      }
      if (kt + 1 < nk) sstore(buf ^ 1);
      __syncthreads();
    }
  } else {
    // tile t lives in buffer t % 3; tile t+2 is loaded during step t and
    // staged at its end; the barrier closing step t-1 published tile t+1 and
    // retired every read of buffer (t+2) % 3.
    if (nk > 0) {
      gload(kbeg);
      sstore(0);
    }
    if (nk > 1) {
      gload(kbeg + BK);
      sstore(1);
    }
    __syncthreads();
    f32x4 fa[TM], fb[TN];
    if (nk > 0) read_frags(smem, 0, fa, fb);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int nxt = cur == 2 ? 0 : cur + 1, stg = nxt == 2 ? 0 : nxt + 1;
      if (kt + 2 < nk) gload(kbeg + (kt + 2) * BK);
      const float* As = smem + cur * STAGE;
      bias_part(As);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 8) {
        f32x4 ga[TM], gb[TN];
        if (kk + 8 < BK) read_frags(As, kk + 8, ga, gb);
        else if (kt + 1 < nk) read_frags(smem + nxt * STAGE, 0, ga, gb);
        mfma_group(fa, fb);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = ga[i];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = gb[j];
      }
      if (kt + 2 < nk) sstore(stg);
      __syncthreads();
      cur = nxt;
    }
  }

  const int hi = lane >> 5;
  if constexpr (P::TILE_EPI) {
    // the TN column tiles of a wave hold, per register, TN values of the same
    // (row, lane column) — e.g. the r/z/n gate pre-activations of one GRU unit
    static_assert(WN == 1, "tile epilogue: one wave column");
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        float v[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) v[j] = acc[i][j][r];
        p.store_tile(m0 + row, blockIdx.y * 32 + frow, z, v);
      }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          const int col = (wn * TN + j) * 32 + frow;
          p.store(m0 + row, n0 + col, z, acc[i][j][r]);
        }
  }
  if constexpr (P::BIAS_FROM_A) {
    if (blockIdx.y == 0) {   // fixed-order combine of the G row-group partials
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

template <int BM_, int BN_, int WM_, int WN_, bool AKC, bool BKC, bool BIASA = false, int BK_ = BK16>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NT = 64 * WM_ * WN_, BK = BK_;
  static constexpr bool A_KC = AKC, B_KC = BKC, BIAS_FROM_A = BIASA, TILE_EPI = false, B_TILE = false;
  struct ACtx { const float* p; int a; int b; bool ok; };
  struct BCtx { const float* p; int a; bool ok; };
};

// u8 operands are staged as exact integers 0..255 (loaders return the raw
// uint32_t, to_f32x4 widens it); the 1/255 of the decode is folded into the
// epilogue (forward) or the slab reduce (wgrad): Σ w·u/255 instead of
// Σ w·fl(u/255), a ≤ 1-ulp-per-term difference (within the fp32 tolerance of
// the GEMM's own summation order) for 16 fewer VALU ops per 4 bytes.

// obs row of minibatch sample b: storage row idx[b] (gather) or row0 + b
__device__ __forceinline__ long long obs_row(const int64_t* idx, long long row0, int b) {
  return idx ? (long long)idx[b] : row0 + b;
}

// Linear + ReLU: out[m][n] = relu(Σ_k x[m][k] w[n][k] + bias[n])
template <class C_>
struct DenseReluFwd : C_ {
  const float* x; const float* w; const float* bias; float* out; int M, N, K;
  int lda = 0, ldo = 0, relu = 1;   // row strides (0: K / N); activation 0 none, 1 ReLU, 2 tanh
  const int64_t* idx = nullptr;      // A-row gather (row idx[m] of x)
  using ACtx = typename C_::ACtx;
  using BCtx = typename C_::BCtx;
  __device__ ACtx a_ctx(int m, int) const {
    if (m >= M) return {x, 0, 0, false};
    return {x + (size_t)(idx ? idx[m] : m) * (lda ? lda : K), 0, 0, true};
  }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    return (c.ok && k < K) ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ BCtx b_ctx(int n, int) const { return {w + (size_t)n * K, 0, n < N}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return (c.ok && k < K) ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = K; }
  __device__ void store(int m, int n, int, float v) const {
    if (m < M && n < N) {
      float y = bias ? v + bias[n] : v;
      out[(size_t)m * (ldo ? ldo : N) + n] = relu == 1 ? fmaxf(y, 0.f) : (relu == 2 ? tanhf(y) : y);
    }
  }
  // vector epilogue (see DenseDgradMask::store4); vec = 1 only with N, ldo and the
  // pointers 16-B compatible
  static constexpr bool VEC_STORE = true;
  int vec = 0;
  __device__ void store4(int m, int n, int, const f32x4& v) const {
    if (m >= M || n >= N) return;
    f32x4 y = v;
    if (bias) y += *reinterpret_cast<const f32x4*>(bias + n);
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = relu == 1 ? fmaxf(y[r], 0.f) : (relu == 2 ? tanhf(y[r]) : y[r]);
    *reinterpret_cast<f32x4*>(out + (size_t)m * (ldo ? ldo : N) + n) = y;
  }
};

// dx[m][n] = (act[m][n] > 0) * Σ_k dy[m][k] wt[n][k]
template <class C_>
struct DenseDgradMask : C_ {
  const float* dy; const float* wt; const float* act; float* dx; int M, N, K;
  int ldact = 0;   // act row stride (0: N); act NULL: no mask
  int mode = 1;    // 1: ReLU mask (act > 0), 2: tanh derivative (1 - act²)
  using ACtx = typename C_::ACtx;
  using BCtx = typename C_::BCtx;
  __device__ ACtx a_ctx(int m, int) const { return {dy + (size_t)m * K, 0, 0, m < M}; }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    return (c.ok && k < K) ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ BCtx b_ctx(int n, int) const { return {wt + (size_t)n * K, 0, n < N}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return (c.ok && k < K) ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = K; }
  __device__ void store(int m, int n, int, float v) const {
    if (m < M && n < N) {
      const size_t i = (size_t)m * N + n;
      if (!act) {
        dx[i] = v;
      } else {
        const float y = act[(size_t)m * (ldact ? ldact : N) + n];
        dx[i] = mode == 2 ? v * (1.0f - y * y) : (y > 0.f ? v : 0.f);
      }
    }
  }
  // vector epilogue (igemm_x9_kernel, vec = 1 set by the launcher when N, the act row
  // stride and both pointers allow 16-B accesses): columns n .. n + 3 of row m
  static constexpr bool VEC_STORE = true;
  int vec = 0;
  __device__ void store4(int m, int n, int, const f32x4& v) const {
    if (m >= M || n >= N) return;
    f32x4 o = v;
    if (act) {
      const f32x4 y = *reinterpret_cast<const f32x4*>(act + (size_t)m * (ldact ? ldact : N) + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = mode == 2 ? v[r] * (1.0f - y[r] * y[r]) : (y[r] > 0.f ? v[r] : 0.f);
    }
    *reinterpret_cast<f32x4*>(dx + (size_t)m * N + n) = o;
  }
};

// A operand (row m, k) by branch-free buffer loads (see DenseWgradB): byte offset
// m·ld·4 + k·4 in one resource over rows [0, M); a row past M starts out of range
// (0x80000000) and k ≥ K is sent there by a select, so each load is one v_cndmask
// instead of an exec-mask branch and a 64-bit address.  The launcher checks
// M·ld·4 < 2^31 (and that there is no row gather).
struct ABufCtx { uint32_t off; };
__device__ __forceinline__ f32x4 abuf_load(const float* base, uint32_t bytes, const ABufCtx& c, int k, int K) {
  const uint32_t off = k < K ? c.off + 4u * (uint32_t)k : 0x80000000u;
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(base, bytes), off, 0, 0));
}

template <class C_>
struct DenseReluFwdB : DenseReluFwd<C_> {
  using ACtx = ABufCtx;
  __device__ uint32_t ld() const { return (uint32_t)(this->lda ? this->lda : this->K); }
  __device__ ACtx a_ctx(int m, int) const { return {m < this->M ? 4u * (uint32_t)m * ld() : 0x80000000u}; }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    return abuf_load(this->x, 4u * (uint32_t)this->M * ld(), c, k, this->K);
  }
};

template <class C_>
struct DenseDgradMaskB : DenseDgradMask<C_> {
  using ACtx = ABufCtx;
  __device__ ACtx a_ctx(int m, int) const { return {m < this->M ? 4u * (uint32_t)m * (uint32_t)this->K : 0x80000000u}; }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    return abuf_load(this->dy, 4u * (uint32_t)this->M * (uint32_t)this->K, c, k, this->K);
  }
};

template <class C_>
struct WgradBase : C_ {
  const float* dz; int COUT; long long R; int chunk;  // chunk: multiple of 16 (and of BK)
  float* slab; float* slab_bias; int NW;             // slab [Z][COUT][NW]
  using ACtx = typename C_::ACtx;
  __device__ ACtx a_ctx(int co, int) const { return {dz + co, 0, 0, co < COUT}; }
  __device__ f32x4 a_load(const ACtx& c, int r) const {
    return (c.ok && r < R) ? *reinterpret_cast<const f32x4*>(c.p + (size_t)r * COUT) : zero4();
  }
  __device__ void k_range(int z, int& b, int& e) const {
    const long long bb = (long long)z * chunk;
    b = (int)(bb < R ? bb : R);
    const long long ee = bb + chunk;
    e = (int)(ee < R ? ee : R);
  }
  __device__ void store(int m, int n, int z, float v) const {
    if (m < COUT && n < NW) slab[((size_t)z * COUT + m) * NW + n] = v;
  }
  static constexpr bool VEC_STORE = true;   // vec = 1: NW % 4 == 0, 16-B aligned slab
  int vec = 0;
  __device__ void store4(int m, int n, int z, const f32x4& v) const {
    if (m < COUT && n < NW) *reinterpret_cast<f32x4*>(slab + ((size_t)z * COUT + m) * NW + n) = v;
  }
  __device__ void store_bias(int m, int z, float v) const {
    if (m < COUT) slab_bias[(size_t)z * COUT + m] = v;
  }
};

// Linear wgrad: X(r, kk) = x[r][kk]
template <class C_>
struct DenseWgrad : WgradBase<C_> {
  const float* x; int K;
  struct BCtx { const float* p; bool ok; };
  __device__ BCtx b_ctx(int n, int) const { return {x + n, n < K}; }
  __device__ f32x4 b_load(const BCtx& c, int r) const {
    return (c.ok && r < this->R) ? *reinterpret_cast<const f32x4*>(c.p + (size_t)r * K) : zero4();
  }
};

// Linear wgrad with branch-free buffer loads (the split-at-staging fc / GRU weight
// gradients): operand row r, column c at byte offset c·4 + r·ld·4 of one buffer
// resource over the whole operand; rows past R read 0 from beyond the resource's
// range and a column past the width starts out of range (0x80000000), so no load
// needs an exec-mask branch or a 64-bit address (DenseWgrad's 16 loads per k-step
// compiled to a branch and a 64-bit multiply each).  Offsets are 32-bit: the
// launcher checks R·width·4 < 2^31.
template <class C_>
struct DenseWgradB : WgradBase<C_> {
  const float* x; int K;
  struct ACtx { uint32_t off; };
  struct BCtx { uint32_t off; };
  __device__ ACtx a_ctx(int co, int) const { return {co < this->COUT ? 4u * (uint32_t)co : 0x80000000u}; }
  __device__ f32x4 a_load(const ACtx& c, int r) const {
    const auto rs = make_rsrc(this->dz, (uint32_t)(this->R * this->COUT) * 4u);
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         rs, c.off + __umul24((uint32_t)r, 4u * (uint32_t)this->COUT), 0, 0));
  }
  __device__ BCtx b_ctx(int n, int) const { return {n < K ? 4u * (uint32_t)n : 0x80000000u}; }
  __device__ f32x4 b_load(const BCtx& c, int r) const {
    const auto rs = make_rsrc(x, (uint32_t)(this->R * K) * 4u);
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         rs, c.off + __umul24((uint32_t)r, 4u * (uint32_t)K), 0, 0));
  }
};

// Deterministic column sums: out[c] = scale * Σ_z src[z*ld + c], c < cols.
// A block covers 32 consecutive columns with 8 z-groups (each summing
// z ≡ g mod 8 in a fixed order, 4 loads in flight), then combines the groups
// in a fixed order — bitwise reproducible, and ≥ cols/32 blocks of parallelism.
//   map kind 0: w[c]                                  (conv1 (c,ky,kx), biases)
//   map kind 1: c=(m, n=(ky,kx,ci)) -> w[m][ci][ky][kx]  (conv2/conv3; a=KS, b=CIN, nw)
//   map kind 2: c=(m, n=(p,ch))     -> w[m][ch*P + p]    (fc; a=C, b=P, nw)
//   map kind 3: c=(m, n) -> w[m][n] for n < a, dropped for n >= a (K padding; a=width, nw)
struct ColMap {
  int kind, a, b, nw;
  __device__ __forceinline__ size_t operator()(long long c) const {
    if (kind == 0) return (size_t)c;
    const int m = (int)(c / nw), n = (int)(c - (long long)m * nw);
    if (kind == 3) return n < a ? (size_t)m * a + n : (size_t)-1;
    if (kind == 1) {
      const int ky = n / (a * b), rem = n - ky * (a * b), kx = rem / b, ci = rem - kx * b;
      return (size_t)m * nw + (size_t)ci * a * a + ky * a + kx;
    }
    const int pp = n / a, ch = n - pp * a;
    return (size_t)m * nw + (size_t)ch * b + pp;
  }
};

__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ src, long long ld, int Z,
                                                     long long cols, ColMap map, float* __restrict__ out, float scale,
                                                     int accumulate) {
  const int cl = threadIdx.x & 31, zg = threadIdx.x >> 5;
  const long long c = (long long)blockIdx.x * 32 + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < cols) {
    const float* p = src + c;
    int z = zg;
    for (; z + 24 < Z; z += 32) {
      s0 += p[(size_t)z * ld];
      s1 += p[(size_t)(z + 8) * ld];
      s2 += p[(size_t)(z + 16) * ld];
      s3 += p[(size_t)(z + 24) * ld];
    }
    for (; z < Z; z += 8) s0 += p[(size_t)z * ld];
  }
  __shared__ float red[8][33];
  red[zg][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (zg == 0 && c < cols) {
    float t = red[0][cl];
#pragma unroll
    for (int g = 1; g < 8; ++g) t += red[g][cl];
    t *= scale;
    const size_t o = map(c);
    if (o != (size_t)-1) out[o] = accumulate ? out[o] + t : t;
  }
}

// flops: algorithmic FLOPs of this launch (2·M·N·K of the GEMM it computes)
template <class P>
int launch(const P& p, long long M, int N, int Z, hipStream_t st, const char* name, double flops) {
  if (M <= 0 || N <= 0 || Z <= 0) return 0;
  const long long gx = (M + P::BM - 1) / P::BM;
  if (gx > 0x7fffffffLL) {
    ppo_set_error("%s: grid too large (M=%lld)", name, M);
    return PPO_ESHAPE;
  }
  dim3 grid((unsigned)gx, (unsigned)((N + P::BN - 1) / P::BN), (unsigned)Z);
  int slot;
  const bool prof = ppo_prof_begin(name, st, &slot);
  igemm_kernel<P><<<grid, P::NT, 0, st>>>(p);
  if (prof) ppo_prof_end(slot, st, flops);
  PPO_LAUNCH_CHECK(name);
  return 0;
}


static inline int colsum(const float* src, long long ld, int Z, long long cols, ColMap map, float* out, float scale,
                         int accumulate, hipStream_t st) {
  if (cols <= 0) return 0;
  colsum_kernel<<<ceil_div(cols, 32), 256, 0, st>>>(src, ld, Z, cols, map, out, scale, accumulate);
  PPO_LAUNCH_CHECK("colsum_kernel");
  return 0;
}

}  // namespace
