// CNNBase trunk on fp32 MFMA (v_mfma_f32_32x32x2_f32): forward (K7-K10),
// input-gradient (dgrad) and weight-gradient (wgrad) passes of K16.
//
// Reference network: CNNBase (ppo-dash-study/001_baseline/ppo/model.py:169-199,
// = ppo-dash-training/.../a2c_ppo_acktr/model.py:169-199):
//   conv1 Conv2d(C,32,8,s4)+ReLU -> conv2 Conv2d(32,64,4,s2)+ReLU ->
//   conv3 Conv2d(64,32,3,s1)+ReLU -> Flatten -> Linear(1568,H)+ReLU
// The reference runs these as cuDNN/MKL calls plus autograd; here every pass is
// an implicit GEMM with the im2col gather folded into the operand loader, the
// bias + ReLU (forward) or ReLU-mask (dgrad) folded into the epilogue, and the
// minibatch row gather (feed_forward_generator `[indices]`, storage.py:143)
// folded into conv1's loader — no im2col or gathered-obs buffer ever exists.
//
// Activation layout in HBM: NHWC fp32 ([B][H][W][C]), so an im2col row's k
// index (ky, kx, ci) reads 16 contiguous bytes per float4.  The observation is
// the storage's u8 NCHW plane; its decode (u8/255, IEEE-exact) runs in the
// loader.  Weights are re-packed once per optimizer step (ppo_pack_weights)
// into the k orders the loaders use; gradients are written back in torch order.
//
// MFMA fragment map (guide §3): lane l supplies A[l&31][k=l>>5] and
// B[k=l>>5][l&31].  Tiles sit in LDS either k-contiguous ([rows][BK+4], read as
// one ds_read_b128 of 4 k values per lane) or row-contiguous ([BK][rows], read
// as 4 ds_read_b32); the 4 k values of a lane feed 4 successive MFMAs, so the
// physical k order inside a BK=16 step is a fixed permutation common to A and B.
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
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

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

  f32x4 ra[NVA], rb[NVB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NVA; ++i) ra[i] = aon[i] ? p.a_load(actx[i], k0 + ak[i]) : zero4();
#pragma unroll
    for (int i = 0; i < NVB; ++i) rb[i] = bon[i] ? p.b_load(bctx[i], k0 + bk[i]) : zero4();
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * STAGE;
    float* Bs = As + TA::SIZE;
#pragma unroll
    for (int i = 0; i < NVA; ++i)
      if (aon[i]) *reinterpret_cast<f32x4*>(As + aoff[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < NVB; ++i)
      if (bon[i]) *reinterpret_cast<f32x4*>(Bs + boff[i]) = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float bias_acc = 0.f;

  if (nk > 0) {
    gload(kbeg);
    sstore(0);
  }
  __syncthreads();
  const int frow = lane & 31, fk = 4 * (lane >> 5);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kbeg + (kt + 1) * BK);
    const float* As = smem + buf * STAGE;
    const float* Bs = As + TA::SIZE;
    if constexpr (P::BIAS_FROM_A) {
      static_assert(!P::A_KC, "bias partials read the row-contiguous A tile");
      if (blockIdx.y == 0 && tid < BM) {
#pragma unroll
        for (int k = 0; k < BK; ++k) bias_acc += As[k * BM + tid];
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 8) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<BM, P::A_KC, BK>(As, (wm * TM + i) * 32 + frow, kk + fk);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = frag<BN, P::B_KC, BK>(Bs, (wn * TN + j) * 32 + frow, kk + fk);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  const int hi = lane >> 5;
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
  if constexpr (P::BIAS_FROM_A) {
    if (blockIdx.y == 0 && tid < BM) p.store_bias(m0 + tid, z, bias_acc);
  }
}

template <int BM_, int BN_, int WM_, int WN_, bool AKC, bool BKC, bool BIASA = false, int BK_ = BK16>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NT = 64 * WM_ * WN_, BK = BK_;
  static constexpr bool A_KC = AKC, B_KC = BKC, BIAS_FROM_A = BIASA;
  struct ACtx { const float* p; int a; int b; bool ok; };
  struct BCtx { const float* p; int a; bool ok; };
};

// u8 operand as exact integers 0..255; the 1/255 of the decode is folded into
// the epilogue (forward) or the slab reduce (wgrad): Σ w·u/255 instead of
// Σ w·fl(u/255), a ≤ 1-ulp-per-term difference (within the fp32 tolerance of
// the GEMM's own summation order) for 16 fewer VALU ops per 4 bytes.
__device__ __forceinline__ f32x4 u8x4(uint32_t u) {
  return f32x4{(float)(u & 255u), (float)((u >> 8) & 255u), (float)((u >> 16) & 255u), (float)(u >> 24)};
}

// obs row of minibatch sample b: storage row idx[b] (gather) or row0 + b
__device__ __forceinline__ long long obs_row(const int64_t* idx, long long row0, int b) {
  return idx ? (long long)idx[b] : row0 + b;
}

// ---------------------------------------------------------------------------
// Forward problems
// ---------------------------------------------------------------------------
constexpr int IMG = 84, IMG2 = 84 * 84;

// conv1: 8x8 stride 4 over the u8/f32 NCHW observation, k = (c, ky, kx) (torch order)
template <typename InT, class C_>
struct Conv1Fwd : C_ {
  using BCtx = typename C_::BCtx;
  const InT* obs; const int64_t* idx; long long row0; int C, M;
  const float* w; const float* bias; float* out;
  struct ACtx { const InT* base; bool ok; };
  __device__ ACtx a_ctx(int m, int) const {
    if (m >= M) return {obs, false};
    const int b = m / 400, pp = m - b * 400, oy = pp / 20, ox = pp - oy * 20;
    return {obs + obs_row(idx, row0, b) * (long long)(C * IMG2) + (oy * 4) * IMG + ox * 4, true};
  }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    if (!c.ok) return zero4();
    const int ch = k >> 6, ky = (k >> 3) & 7, kx = k & 7;
    const InT* q = c.base + ch * IMG2 + ky * IMG + kx;
    if constexpr (sizeof(InT) == 1) return u8x4(*reinterpret_cast<const uint32_t*>(q));
    else return *reinterpret_cast<const f32x4*>(q);
  }
  __device__ BCtx b_ctx(int n, int) const { return {w + n * (C * 64), 0, n < 32}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = C * 64; }
  __device__ void store(int m, int n, int, float v) const {
    if constexpr (sizeof(InT) == 1) v *= (1.0f / 255.0f);
    if (m < M) out[(size_t)m * 32 + n] = fmaxf(v + bias[n], 0.f);
  }
};

// NHWC conv (conv2, conv3): k = (ky, kx, ci), weights packed [COUT][K]
template <int HIN, int CIN, int KS, int ST, int HOUT, int COUT, class C_>
struct ConvFwd : C_ {
  static constexpr int K = KS * KS * CIN, P = HOUT * HOUT;
  const float* in; const float* w; const float* bias; float* out; int M;
  using ACtx = typename C_::ACtx;
  using BCtx = typename C_::BCtx;
  __device__ ACtx a_ctx(int m, int) const {
    if (m >= M) return {in, 0, 0, false};
    const int b = m / P, pp = m - b * P, oy = pp / HOUT, ox = pp - oy * HOUT;
    return {in + ((size_t)(b * HIN + ST * oy) * HIN + ST * ox) * CIN, 0, 0, true};
  }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    if (!c.ok) return zero4();
    const int ky = k / (KS * CIN), rem = k - ky * (KS * CIN), kx = rem / CIN, ci = rem - kx * CIN;
    return *reinterpret_cast<const f32x4*>(c.p + (ky * HIN + kx) * CIN + ci);
  }
  __device__ BCtx b_ctx(int n, int) const { return {w + (size_t)n * K, 0, n < COUT}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = K; }
  __device__ void store(int m, int n, int, float v) const {
    if (m < M && n < COUT) out[(size_t)m * COUT + n] = fmaxf(v + bias[n], 0.f);
  }
};

// Linear + ReLU: out[m][n] = relu(Σ_k x[m][k] w[n][k] + bias[n])
template <class C_>
struct DenseReluFwd : C_ {
  const float* x; const float* w; const float* bias; float* out; int M, N, K;
  using ACtx = typename C_::ACtx;
  using BCtx = typename C_::BCtx;
  __device__ ACtx a_ctx(int m, int) const { return {x + (size_t)m * K, 0, 0, m < M}; }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    return (c.ok && k < K) ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ BCtx b_ctx(int n, int) const { return {w + (size_t)n * K, 0, n < N}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return (c.ok && k < K) ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = K; }
  __device__ void store(int m, int n, int, float v) const {
    if (m < M && n < N) out[(size_t)m * N + n] = fmaxf(v + bias[n], 0.f);
  }
};

// ---------------------------------------------------------------------------
// Input-gradient (dgrad) problems; epilogue applies the ReLU mask of the
// layer below (threshold_backward: pass where the saved output is > 0).
// ---------------------------------------------------------------------------
// dx[m][n] = (act[m][n] > 0) * Σ_k dy[m][k] wt[n][k]
template <class C_>
struct DenseDgradMask : C_ {
  const float* dy; const float* wt; const float* act; float* dx; int M, N, K;
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
      dx[i] = act[i] > 0.f ? v : 0.f;
    }
  }
};

// stride-1 conv dgrad (conv3): m = (b, y, x) input pixel, n = ci,
// k = (ky, kx, co): dy[b][y-ky][x-kx][co] (0 outside), wd packed [CIN][K]
template <int HIN, int CIN, int KS, int HOUT, int COUT, class C_>
struct ConvDgradS1 : C_ {
  static constexpr int K = KS * KS * COUT, PIN = HIN * HIN;
  const float* dy; const float* wd; const float* act; float* dx; int M;
  struct ACtx { const float* p; int y; int x; bool ok; };
  using BCtx = typename C_::BCtx;
  __device__ ACtx a_ctx(int m, int) const {
    if (m >= M) return {dy, 0, 0, false};
    const int b = m / PIN, pp = m - b * PIN, y = pp / HIN, x = pp - y * HIN;
    return {dy + (size_t)b * HOUT * HOUT * COUT, y, x, true};
  }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    const int ky = k / (KS * COUT), rem = k - ky * (KS * COUT), kx = rem / COUT, co = rem - kx * COUT;
    const int oy = c.y - ky, ox = c.x - kx;
    if (!c.ok || oy < 0 || oy >= HOUT || ox < 0 || ox >= HOUT) return zero4();
    return *reinterpret_cast<const f32x4*>(c.p + (oy * HOUT + ox) * COUT + co);
  }
  __device__ BCtx b_ctx(int n, int) const { return {wd + (size_t)n * K, 0, n < CIN}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = K; }
  __device__ void store(int m, int n, int, float v) const {
    if (m < M && n < CIN) {
      const size_t i = (size_t)m * CIN + n;
      dx[i] = act[i] > 0.f ? v : 0.f;
    }
  }
};

// conv2 dgrad (4x4 stride 2, 20x20 <- 9x9): split by output-pixel phase
// (y&1, x&1) = blockIdx.z so each phase is a dense 2x2-tap problem:
// m = (b, yy, xx) with y = 2yy+py; k = (ty, tx, co): ky = py+2ty,
// oy = yy - ty.  wd packed [4 phases][CIN][4*COUT].
template <class C_>
struct Conv2Dgrad : C_ {
  using BCtx = typename C_::BCtx;
  static constexpr int HIN = 20, CIN = 32, HOUT = 9, COUT = 64, K = 4 * COUT, PPH = 100;
  const float* dy; const float* wd; const float* act; float* dx; int M;  // M = B*100 per phase
  struct ACtx { const float* p; int yy; int xx; bool ok; };
  __device__ ACtx a_ctx(int m, int) const {
    if (m >= M) return {dy, 0, 0, false};
    const int b = m / PPH, pp = m - b * PPH, yy = pp / 10, xx = pp - yy * 10;
    return {dy + (size_t)b * HOUT * HOUT * COUT, yy, xx, true};
  }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    const int ty = k >> 7, tx = (k >> 6) & 1, co = k & 63;
    const int oy = c.yy - ty, ox = c.xx - tx;
    if (!c.ok || oy < 0 || oy >= HOUT || ox < 0 || ox >= HOUT) return zero4();
    return *reinterpret_cast<const f32x4*>(c.p + (oy * HOUT + ox) * COUT + co);
  }
  __device__ BCtx b_ctx(int n, int z) const { return {wd + ((size_t)z * CIN + n) * K, 0, n < CIN}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = K; }
  __device__ void store(int m, int n, int z, float v) const {
    if (m < M && n < CIN) {
      const int b = m / PPH, pp = m - b * PPH, yy = pp / 10, xx = pp - yy * 10;
      const int y = 2 * yy + (z >> 1), x = 2 * xx + (z & 1);
      const size_t i = ((size_t)(b * HIN + y) * HIN + x) * CIN + n;
      dx[i] = act[i] > 0.f ? v : 0.f;
    }
  }
};

// ---------------------------------------------------------------------------
// Weight-gradient (wgrad) problems: dW[co][kk] = Σ_r dz[r][co] · X(r, kk)
// over the reduction r = (b, output pixel), split over blockIdx.z into fp32
// partial slabs (deterministic sum in ppo_wgrad_reduce).  Both operands are
// row-contiguous tiles; blocks of tile column 0 also sum the dz tile into the
// bias partial (db[co] = Σ_r dz[r][co]).
// ---------------------------------------------------------------------------
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
  __device__ void store_bias(int m, int z, float v) const {
    if (m < COUT) slab_bias[(size_t)z * COUT + m] = v;
  }
};

// conv1 wgrad: X(r, kk) = decoded obs[idx[b]][c][4oy+ky][4ox+kx], kk = (c,ky,kx)
template <typename InT, class C_>
struct Conv1Wgrad : WgradBase<C_> {
  const InT* obs; const int64_t* idx; long long row0; int C;
  struct BCtx { int off; bool ok; };
  __device__ BCtx b_ctx(int n, int) const {
    const int ch = n >> 6, ky = (n >> 3) & 7, kx = n & 7;
    return {ch * IMG2 + ky * IMG + kx, n < C * 64};
  }
  __device__ f32x4 b_load(const BCtx& c, int r) const {
    if (!c.ok || r >= this->R) return zero4();
    const int b = r / 400, pp = r - b * 400, oy = pp / 20, ox = pp - oy * 20;
    const InT* q = obs + obs_row(idx, row0, b) * (long long)(C * IMG2) + (oy * 4) * IMG + ox * 4 + c.off;
    if constexpr (sizeof(InT) == 1) return u8x4(*reinterpret_cast<const uint32_t*>(q));
    else return *reinterpret_cast<const f32x4*>(q);
  }
};

// NHWC conv wgrad (conv2, conv3): kk = (ky, kx, ci)
template <int HIN, int CIN, int KS, int ST, int HOUT, class C_>
struct ConvWgrad : WgradBase<C_> {
  static constexpr int K = KS * KS * CIN, P = HOUT * HOUT;
  const float* in;
  struct BCtx { int off; bool ok; };
  __device__ BCtx b_ctx(int n, int) const {
    const int ky = n / (KS * CIN), rem = n - ky * (KS * CIN), kx = rem / CIN, ci = rem - kx * CIN;
    return {(ky * HIN + kx) * CIN + ci, n < K};
  }
  __device__ f32x4 b_load(const BCtx& c, int r) const {
    if (!c.ok || r >= this->R) return zero4();
    const int b = r / P, pp = r - b * P, oy = pp / HOUT, ox = pp - oy * HOUT;
    return *reinterpret_cast<const f32x4*>(in + ((size_t)(b * HIN + ST * oy) * HIN + ST * ox) * CIN + c.off);
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

// Deterministic column sums: out[c] = scale * Σ_z src[z*ld + c], c < cols.
// A block covers 32 consecutive columns with 8 z-groups (each summing
// z ≡ g mod 8 in a fixed order, 4 loads in flight), then combines the groups
// in a fixed order — bitwise reproducible, and ≥ cols/32 blocks of parallelism.
//   map kind 0: w[c]                                  (conv1 (c,ky,kx), biases)
//   map kind 1: c=(m, n=(ky,kx,ci)) -> w[m][ci][ky][kx]  (conv2/conv3; a=KS, b=CIN, nw)
//   map kind 2: c=(m, n=(p,ch))     -> w[m][ch*P + p]    (fc; a=C, b=P, nw)
struct ColMap {
  int kind, a, b, nw;
  __device__ __forceinline__ size_t operator()(long long c) const {
    if (kind == 0) return (size_t)c;
    const int m = (int)(c / nw), n = (int)(c - (long long)m * nw);
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
    out[o] = accumulate ? out[o] + t : t;
  }
}

// Pack torch-layout weights into the loaders' k orders (once per optimizer step).
//   W2p [64][512]  (ky,kx,ci)       W3p [32][576] (ky,kx,ci)
//   W4p [H][1568]  (p,c)            W4T [1568][H] (p,c) x n
//   W3d [64][288]  ci x (ky,kx,co)  W2d [4][32][256] phase x ci x (ty,tx,co)
__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ w2, const float* __restrict__ w3,
                                                           const float* __restrict__ w4, int H,
                                                           float* __restrict__ out) {
  const long long n2 = 64 * 512, n3 = 32 * 576, n4 = (long long)H * 1568, n3d = 64 * 288, n2d = 4 * 32 * 256;
  const long long total = n2 + n3 + 2 * n4 + n3d + n2d;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    long long j = i;
    float v;
    if (j < n2) {
      const int co = (int)(j / 512), k = (int)(j % 512), ky = k / 128, kx = (k / 32) % 4, ci = k % 32;
      v = w2[co * 512 + ci * 16 + ky * 4 + kx];
    } else if ((j -= n2) < n3) {
      const int co = (int)(j / 576), k = (int)(j % 576), ky = k / 192, kx = (k / 64) % 3, ci = k % 64;
      v = w3[co * 576 + ci * 9 + ky * 3 + kx];
    } else if ((j -= n3) < n4) {
      const long long n = j / 1568;
      const int k = (int)(j % 1568), pp = k / 32, c = k % 32;
      v = w4[n * 1568 + c * 49 + pp];
    } else if ((j -= n4) < n4) {
      const int k = (int)(j / H), n = (int)(j % H), pp = k / 32, c = k % 32;
      v = w4[(long long)n * 1568 + c * 49 + pp];
    } else if ((j -= n4) < n3d) {
      const int ci = (int)(j / 288), k = (int)(j % 288), ky = k / 96, kx = (k / 32) % 3, co = k % 32;
      v = w3[co * 576 + ci * 9 + ky * 3 + kx];
    } else {
      j -= n3d;
      const int ph = (int)(j / 8192), rem = (int)(j % 8192), ci = rem / 256, k = rem % 256;
      const int ty = k >> 7, tx = (k >> 6) & 1, co = k & 63;
      const int ky = (ph >> 1) + 2 * ty, kx = (ph & 1) + 2 * tx;
      v = w2[co * 512 + ci * 16 + ky * 4 + kx];
    }
    out[i] = v;
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

using CfgN32 = Cfg<256, 32, 4, 1, true, true>;
using CfgN64 = Cfg<128, 64, 2, 2, true, true>;
using CfgN128 = Cfg<128, 128, 2, 2, true, true>;
using CfgN64s = Cfg<256, 64, 4, 1, true, true>;

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
PPO_API long long ppo_packed_weights_size(int H) {
  return 64LL * 512 + 32 * 576 + 2LL * H * 1568 + 64 * 288 + 4 * 32 * 256;
}

// offsets (floats) of the packed segments inside the pack buffer
PPO_API int ppo_packed_offsets(int H, long long* off6) {
  off6[0] = 0;                         // W2p
  off6[1] = off6[0] + 64 * 512;        // W3p
  off6[2] = off6[1] + 32 * 576;        // W4p
  off6[3] = off6[2] + (long long)H * 1568;  // W4T
  off6[4] = off6[3] + (long long)H * 1568;  // W3d
  off6[5] = off6[4] + 64 * 288;        // W2d
  return 0;
}

PPO_API int ppo_pack_weights(const float* w2, const float* w3, const float* w4, int H, float* packed, void* stream) {
  PPO_REQUIRE(H > 0 && H % 4 == 0, "ppo_pack_weights: hidden size %d must be a positive multiple of 4", H);
  const long long total = ppo_packed_weights_size(H);
  long long b = (total + 255) / 256;
  pack_weights_kernel<<<(unsigned)(b < 2048 ? b : 2048), 256, 0, as_stream(stream)>>>(w2, w3, w4, H, packed);
  PPO_LAUNCH_CHECK("pack_weights_kernel");
  return 0;
}

// ---------------------------------------------------------------------------
// Tile-configuration variants (A/B knobs for tools/kbench.py; defaults are the
// measured best on MI355X).  ppo_tune_set("conv1_fwd", v) etc.
// ---------------------------------------------------------------------------
enum { TK_CONV1_FWD, TK_CONV3_FWD, TK_CONV2_DGRAD, TK_CONV3_DGRAD, TK_CONV1_WGRAD, TK_N };
static const char* g_tune_names[TK_N] = {"conv1_fwd", "conv3_fwd", "conv2_dgrad", "conv3_dgrad", "conv1_wgrad"};
static int g_tune[TK_N] = {1, 1, 1, 1, 1};  // measured best (kbench sweep, profiles/)

PPO_API int ppo_tune_set(const char* key, int value) {
  for (int i = 0; i < TK_N; ++i)
    if (strcmp(key, g_tune_names[i]) == 0) {
      g_tune[i] = value;
      return 0;
    }
  ppo_set_error("ppo_tune_set: unknown key %s", key);
  return PPO_EARG;
}

// N = 32 output-channel problems (conv1/conv3 fwd, conv2 dgrad)
using V32_0 = Cfg<256, 32, 4, 1, true, true>;           // 4 waves x 64 rows, 46 KB LDS
using V32_1 = Cfg<128, 32, 4, 1, true, true>;           // 4 waves x 32 rows, 26 KB
using V32_2 = Cfg<128, 32, 2, 1, true, true>;           // 2 waves x 64 rows, 26 KB
using V32_3 = Cfg<128, 32, 4, 1, true, true, false, 32>;  // BK 32, 46 KB
using V32_4 = Cfg<64, 32, 2, 1, true, true, false, 32>;   // 2 waves x 32 rows, BK 32, 28 KB
// N = 64 problems (conv2 fwd, conv3 dgrad)
using V64_0 = Cfg<128, 64, 2, 2, true, true>;
using V64_1 = Cfg<64, 64, 2, 2, true, true>;
using V64_2 = Cfg<128, 64, 4, 1, true, true>;

#define PPO_VARIANTS32(TEMPL, SETUP, M, N, Z, NAME, FLOPS)                                        \
  switch (g_tune[tk]) {                                                                           \
    case 1: { TEMPL(V32_1) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
    case 2: { TEMPL(V32_2) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
    case 3: { TEMPL(V32_3) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
    case 4: { TEMPL(V32_4) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
    default: { TEMPL(V32_0) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
  }

#define PPO_VARIANTS64(TEMPL, SETUP, M, N, Z, NAME, FLOPS)                                        \
  switch (g_tune[tk]) {                                                                           \
    case 1: { TEMPL(V64_1) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
    case 2: { TEMPL(V64_2) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
    default: { TEMPL(V64_0) p; SETUP; return launch(p, M, N, Z, as_stream(stream), NAME, FLOPS); } \
  }

// conv1 forward: out [B][20][20][32] = relu(conv(obs rows, W1 torch layout) + b1)
PPO_API int ppo_conv1_fwd(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                          const float* w1, const float* b1, float* out, void* stream) {
  PPO_REQUIRE(B >= 0 && C > 0, "ppo_conv1_fwd: B=%d C=%d", B, C);
  const long long M = (long long)B * 400;
  const int tk = TK_CONV1_FWD;
  const double fl = 2.0 * M * 32 * C * 64;
#define SETUP1(T_)                                                                                 \
  p.obs = (const T_*)obs; p.idx = idx; p.row0 = row0; p.C = C; p.M = (int)M; p.w = w1; p.bias = b1; p.out = out
  if (obs_is_u8) {
#define T1(C_) Conv1Fwd<uint8_t, C_>
    PPO_VARIANTS32(T1, SETUP1(uint8_t), M, 32, 1, "conv1_fwd_u8", fl)
#undef T1
  }
#define T1(C_) Conv1Fwd<float, C_>
  PPO_VARIANTS32(T1, SETUP1(float), M, 32, 1, "conv1_fwd_f32", fl)
#undef T1
#undef SETUP1
}

PPO_API int ppo_conv2_fwd(const float* a1, int B, const float* w2p, const float* b2, float* out, void* stream) {
  ConvFwd<20, 32, 4, 2, 9, 64, V64_0> p;
  p.in = a1; p.w = w2p; p.bias = b2; p.out = out; p.M = B * 81;
  return launch(p, (long long)B * 81, 64, 1, as_stream(stream), "conv2_fwd", 2.0 * B * 81 * 64 * 512);
}

PPO_API int ppo_conv3_fwd(const float* a2, int B, const float* w3p, const float* b3, float* out, void* stream) {
  const int tk = TK_CONV3_FWD;
#define T3(C_) ConvFwd<9, 64, 3, 1, 7, 32, C_>
  PPO_VARIANTS32(T3, (p.in = a2, p.w = w3p, p.bias = b3, p.out = out, p.M = B * 49), (long long)B * 49, 32, 1,
                 "conv3_fwd", 2.0 * B * 49 * 32 * 576)
#undef T3
}

// Linear + ReLU: out [M][N] = relu(x [M][K] · w [N][K]^T + b)
PPO_API int ppo_linear_relu_fwd(const float* x, int M, int K, const float* w, const float* b, int N, float* out,
                                void* stream) {
  PPO_REQUIRE(K % 4 == 0, "ppo_linear_relu_fwd: K=%d must be a multiple of 4", K);
  if (N % 128 == 0) {
    DenseReluFwd<CfgN128> p;
    p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K;
    return launch(p, M, N, 1, as_stream(stream), "linear_relu_fwd", 2.0 * M * N * K);
  }
  DenseReluFwd<CfgN64> p;
  p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K;
  return launch(p, M, N, 1, as_stream(stream), "linear_relu_fwd", 2.0 * M * N * K);
}

// dx [M][N] = (act > 0) * (dy [M][K] · wt [N][K]^T)
PPO_API int ppo_linear_dgrad_mask(const float* dy, int M, int K, const float* wt, int N, const float* act, float* dx,
                                  void* stream) {
  PPO_REQUIRE(K % 4 == 0, "ppo_linear_dgrad_mask: K=%d must be a multiple of 4", K);
  DenseDgradMask<CfgN128> p;
  p.dy = dy; p.wt = wt; p.act = act; p.dx = dx; p.M = M; p.N = N; p.K = K;
  return launch(p, M, N, 1, as_stream(stream), "linear_dgrad_mask", 2.0 * M * N * K);
}

PPO_API int ppo_conv3_dgrad(const float* dz3, int B, const float* w3d, const float* a2, float* dz2, void* stream) {
  const int tk = TK_CONV3_DGRAD;
#define TD3(C_) ConvDgradS1<9, 64, 3, 7, 32, C_>
  PPO_VARIANTS64(TD3, (p.dy = dz3, p.wd = w3d, p.act = a2, p.dx = dz2, p.M = B * 81), (long long)B * 81, 64, 1,
                 "conv3_dgrad", 2.0 * B * 49 * 32 * 576)
#undef TD3
}

PPO_API int ppo_conv2_dgrad(const float* dz2, int B, const float* w2d, const float* a1, float* dz1, void* stream) {
  const int tk = TK_CONV2_DGRAD;
#define TD2(C_) Conv2Dgrad<C_>
  PPO_VARIANTS32(TD2, (p.dy = dz2, p.wd = w2d, p.act = a1, p.dx = dz1, p.M = B * 100), (long long)B * 100, 32, 4,
                 "conv2_dgrad", 2.0 * B * 81 * 64 * 512)
#undef TD2
}

// split count and chunk for a wgrad reduction of R rows (BK-aligned chunks)
PPO_API int ppo_wgrad_splits(long long R, int tiles, int target_blocks, int min_ktiles) {
  long long kt = (R + BK16 - 1) / BK16;
  long long z = target_blocks / (tiles > 0 ? tiles : 1);
  if (z < 1) z = 1;
  if (kt / z < min_ktiles) z = kt / min_ktiles;
  if (z < 1) z = 1;
  if (z > 4096) z = 4096;
  return (int)z;
}

static inline int wgrad_chunk(long long R, int Z) {
  long long kt = (R + BK16 - 1) / BK16;
  return (int)(((kt + Z - 1) / Z) * BK16);
}

template <class P>
static void set_wgrad(P& p, const float* dz, int COUT, long long R, int Z, float* slab, float* slab_bias, int NW) {
  p.dz = dz; p.COUT = COUT; p.R = R; p.chunk = wgrad_chunk(R, Z); p.slab = slab; p.slab_bias = slab_bias; p.NW = NW;
}

using CfgW32 = Cfg<32, 256, 1, 4, false, false, true>;
using CfgW32n = Cfg<32, 128, 1, 4, false, false, true>;
using CfgW64 = Cfg<64, 128, 2, 2, false, false, true>;
using CfgW32b = Cfg<32, 128, 1, 4, false, false, true>;
using CfgWfc = Cfg<128, 128, 2, 2, false, false, true>;

// conv1 wgrad partials: slab [Z][32][C*64], slab_bias [Z][32]
PPO_API int ppo_conv1_wgrad(const float* dz1, const void* obs, int obs_is_u8, const int64_t* idx, long long row0,
                            int C, int B, int Z, float* slab, float* slab_bias, void* stream) {
  const long long R = (long long)B * 400;
  PPO_REQUIRE(R < 0x7fffffffLL, "ppo_conv1_wgrad: B too large");
  const double fl = 2.0 * R * 32 * C * 64;
  if (obs_is_u8) {
    if (g_tune[TK_CONV1_WGRAD] == 1) {
      Conv1Wgrad<uint8_t, CfgW32n> p;
      set_wgrad(p, dz1, 32, R, Z, slab, slab_bias, C * 64);
      p.obs = (const uint8_t*)obs; p.idx = idx; p.row0 = row0; p.C = C;
      return launch(p, 32, C * 64, Z, as_stream(stream), "conv1_wgrad_u8", fl);
    }
    Conv1Wgrad<uint8_t, CfgW32> p;
    set_wgrad(p, dz1, 32, R, Z, slab, slab_bias, C * 64);
    p.obs = (const uint8_t*)obs; p.idx = idx; p.row0 = row0; p.C = C;
    return launch(p, 32, C * 64, Z, as_stream(stream), "conv1_wgrad_u8", fl);
  }
  Conv1Wgrad<float, CfgW32> p;
  set_wgrad(p, dz1, 32, R, Z, slab, slab_bias, C * 64);
  p.obs = (const float*)obs; p.idx = idx; p.row0 = row0; p.C = C;
  return launch(p, 32, C * 64, Z, as_stream(stream), "conv1_wgrad_f32", fl);
}

PPO_API int ppo_conv2_wgrad(const float* dz2, const float* a1, int B, int Z, float* slab, float* slab_bias,
                            void* stream) {
  ConvWgrad<20, 32, 4, 2, 9, CfgW64> p;
  set_wgrad(p, dz2, 64, (long long)B * 81, Z, slab, slab_bias, 512);
  p.in = a1;
  return launch(p, 64, 512, Z, as_stream(stream), "conv2_wgrad", 2.0 * B * 81 * 64 * 512);
}

PPO_API int ppo_conv3_wgrad(const float* dz3, const float* a2, int B, int Z, float* slab, float* slab_bias,
                            void* stream) {
  ConvWgrad<9, 64, 3, 1, 7, CfgW32b> p;
  set_wgrad(p, dz3, 32, (long long)B * 49, Z, slab, slab_bias, 576);
  p.in = a2;
  return launch(p, 32, 576, Z, as_stream(stream), "conv3_wgrad", 2.0 * B * 49 * 32 * 576);
}

// dW[n][k] = Σ_r dy[r][n] x[r][k]: slab [Z][N][K], slab_bias [Z][N]
PPO_API int ppo_linear_wgrad(const float* dy, const float* x, int R, int N, int K, int Z, float* slab,
                             float* slab_bias, void* stream) {
  PPO_REQUIRE(N % 4 == 0 && K % 4 == 0, "ppo_linear_wgrad: N=%d K=%d must be multiples of 4", N, K);
  DenseWgrad<CfgWfc> p;
  set_wgrad(p, dy, N, R, Z, slab, slab_bias, K);
  p.x = x; p.K = K;
  return launch(p, N, K, Z, as_stream(stream), "linear_wgrad", 2.0 * R * N * K);
}

static int colsum(const float* src, long long ld, int Z, long long cols, ColMap map, float* out, float scale,
                  int accumulate, hipStream_t st) {
  if (cols <= 0) return 0;
  colsum_kernel<<<ceil_div(cols, 32), 256, 0, st>>>(src, ld, Z, cols, map, out, scale, accumulate);
  PPO_LAUNCH_CHECK("colsum_kernel");
  return 0;
}

// Σ over the Z split partials (fixed order) -> gw (torch order, see ColMap) and gb
PPO_API int ppo_wgrad_reduce(const float* slab, const float* slab_bias, int Z, int M, int NW, int kind, int a, int b,
                             float* gw, float* gb, float scale, int accumulate, void* stream) {
  PPO_REQUIRE(kind >= 0 && kind <= 2, "ppo_wgrad_reduce: kind=%d", kind);
  hipStream_t st = as_stream(stream);
  const long long cols = (long long)M * NW;
  int rc = colsum(slab, cols, Z, cols, ColMap{kind, a, b, NW}, gw, scale, accumulate, st);
  if (rc) return rc;
  return colsum(slab_bias, M, Z, M, ColMap{0, 0, 0, 1}, gb, 1.0f, accumulate, st);
}

// generic deterministic column sum (used for the heads' partials)
PPO_API int ppo_colsum(const float* src, long long ld, int rows, long long cols, float* out, float scale,
                       int accumulate, void* stream) {
  return colsum(src, ld, rows, cols, ColMap{0, 0, 0, 1}, out, scale, accumulate, as_stream(stream));
}
