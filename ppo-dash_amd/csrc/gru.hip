// Recurrent policy core (K12): the GRU of NNBase, forward and backward
// through time, on the fp32 MFMA implicit-GEMM core.
//
// Reference: NNBase.__init__ / _forward_gru, ppo-dash-training/
// pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/model.py:89-95, 111-166 (torch.nn.GRU,
// gates (r, z, n): r = σ(W_ir x + b_ir + W_hr h + b_hr), z likewise,
// n = tanh(W_in x + b_in + r ⊙ (W_hn h + b_hn)), h' = (1 - z) ⊙ n + z ⊙ h).
// The reference splits the sequence at steps where any env's mask is 0 and
// feeds h·m[start] to each segment; that is exactly h_in(t) = h(t-1)·m(t) at
// every step (the extra ×1 are exact), which is what runs here.
//
// Work split:
//   gi = x · W_ihᵀ + b_ih         one big GEMM over all T·n_env rows (gemm.hip)
//   per step t: gh = h_in · W_hhᵀ and the gate cell fused in the epilogue
//     (tile epilogue: a wave's three 32-column tiles are the r, z, n columns of
//     the same 32 hidden units, so each lane holds all three pre-activations)
//   backward per step (reverse): gate gradients (elementwise) then
//     dh_in = dgh · W_hh with the carry (dh_in + dh'·z)·m(t) in the epilogue
//   after the loop: dW_hh, dW_ih as split-K wgrads over all T·n_env rows,
//     dx = dgi · W_ih[:, :H] masked by the fc ReLU.
// Saved per step for the backward: r, z, n, W_hn h + b_hn, h_in ([T][n][H] each).
#include <mutex>
#include <type_traits>

#include "igemm_x9.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// W_hh products of the register-tiled step kernels on the matrix cores.  Where a
// wave's K run fills whole 32-k steps (BF: the forward for H = 128, 256, 512, the
// BPTT's K halves for H = 128, 256, 512) both operands are split exactly into
// three bf16 parts and the six part products of the convolutions' fp32 emulation
// (DESIGN.md §3, mma9<.., 6>) run on v_mfma_f32_16x16x32_bf16: 6 x 16 cycles per
// 32 k instead of 8 x 32 on v_mfma_f32_16x16x4_f32 (2.7x the rate).  A 32-k step
// takes the lane's own consecutive 16-B chunks 2 kk, 2 kk + 1 (the lane group's k
// of the chunked K order below), for the A and B operands alike, so the sum runs
// over the same k.  Otherwise (H = 64) the exact fp32 MFMAs remain.
template <int KW, bool BF>
struct GruRow {   // one B row of KW k in the chunked K order
  float f[BF ? 1 : KW];
  Frag3 p[BF ? KW / 8 : 1];
};
template <int KW, bool BF>
__device__ __forceinline__ void gru_row_set(const float (&v)[KW], GruRow<KW, BF>& r) {
  if constexpr (BF) {
#pragma unroll
    for (int kk = 0; kk < KW / 8; ++kk)
      split8(f32x4{v[8 * kk], v[8 * kk + 1], v[8 * kk + 2], v[8 * kk + 3]},
             f32x4{v[8 * kk + 4], v[8 * kk + 5], v[8 * kk + 6], v[8 * kk + 7]}, r.p[kk], false);
  } else {
#pragma unroll
    for (int s = 0; s < KW; ++s) r.f[s] = v[s];
  }
}
// acc[rt][g] += a[rt][0 .. KA) · w[g] over its k OFF .. OFF + KA (rt: the block's two
// 16-row tiles); the accumulation order is fixed by (KA, OFF, NG) alone
template <int KA, int OFF, int NG, int KW, bool BF>
__device__ __forceinline__ void gru_mma(const float (&a)[2][KA], const GruRow<KW, BF> (&w)[NG], f32x4 (&acc)[2][NG]) {
  if constexpr (BF) {
    static_assert(KA % 8 == 0 && OFF % 8 == 0, "whole 32-k steps");
#pragma unroll
    for (int kk = 0; kk < KA / 8; ++kk)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        Frag3 fa;
#ifdef GRU_NOSPLIT   // timing anatomy only (wrong results): A's planes without the split VALU
        {
          uint32_t w[4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            w[i] = __builtin_amdgcn_perm(__float_as_uint(a[rt][8 * kk + 2 * i + 1]), __float_as_uint(a[rt][8 * kk + 2 * i]),
                                         0x07060302u);
          fa.h = fa.m = fa.l = __builtin_bit_cast(bf16x8, uint4{w[0], w[1], w[2], w[3]});
        }
#else
        split8(f32x4{a[rt][8 * kk], a[rt][8 * kk + 1], a[rt][8 * kk + 2], a[rt][8 * kk + 3]},
               f32x4{a[rt][8 * kk + 4], a[rt][8 * kk + 5], a[rt][8 * kk + 6], a[rt][8 * kk + 7]}, fa, false);
#endif
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[rt][g] = mma9<false, false, 6>(fa, w[g].p[OFF / 8 + kk], acc[rt][g]);
      }
  } else {
#pragma unroll
    for (int s = 0; s < KA; ++s)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int g = 0; g < NG; ++g)
          acc[rt][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rt][s], w[g].f[OFF + s], acc[rt][g], 0, 0, 0);
  }
}

// gh tile with the fused GRU cell.  B rows n = jt*96 + g*32 + jj <-> W_hh row g*H + jt*32 + jj.
template <class C_>
struct GruStep : C_ {
  static constexpr bool TILE_EPI = true;
  const float* hprev;            // [M][H] h(t-1)
  const float* masks;            // mask plane (NULL: 1)
  const int64_t* mask_idx;       // masks[mask_idx[m]] (NULL: masks[m])
  const float* whh; const float* bhh;
  const float* gi;               // [M][3H] x·W_ihᵀ + b_ih of this step
  float* hout;                   // [M][H]
  float *sr, *sz, *sn, *sghn, *shin;  // saved for backward (NULL: inference)
  int M, H;
  struct ACtx { const float* p; float m; bool ok; };
  using BCtx = typename C_::BCtx;
  __device__ float mask_of(int m) const {
    if (!masks) return 1.0f;
    return masks[mask_idx ? mask_idx[m] : m];
  }
  __device__ ACtx a_ctx(int m, int) const {
    if (m >= M) return {hprev, 0.f, false};
    return {hprev + (size_t)m * H, mask_of(m), true};
  }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    if (!c.ok) return zero4();
    return *reinterpret_cast<const f32x4*>(c.p + k) * c.m;
  }
  __device__ BCtx b_ctx(int n, int) const {
    const int jt = n / 96, rem = n - jt * 96, g = rem >> 5, jj = rem & 31;
    const int j = jt * 32 + jj;
    return {whh + ((size_t)g * H + j) * H, 0, j < H};
  }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = H; }
  __device__ void store(int, int, int, float) const {}
  __device__ void store_tile(int m, int j, int, const float (&v)[3]) const {
    if (m >= M || j >= H) return;
    const float* g = gi + (size_t)m * 3 * H;
    const float ghr = v[0] + bhh[j], ghz = v[1] + bhh[H + j], ghn = v[2] + bhh[2 * H + j];
    const float r = sigm(g[j] + ghr);
    const float z = sigm(g[H + j] + ghz);
    const float n = tanhf(g[2 * H + j] + r * ghn);
    const float hin = hprev[(size_t)m * H + j] * mask_of(m);
    const size_t o = (size_t)m * H + j;
    hout[o] = (1.0f - z) * n + z * hin;
    if (sr) {
      sr[o] = r;
      sz[o] = z;
      sn[o] = n;
      sghn[o] = ghn;
      shin[o] = hin;
    }
  }
};

// dh_in = dgh · W_hh (B = W_hhᵀ packed [H][3H]); carry = (dh_in + dh'·z) · m(t)
template <class C_>
struct GruBwdStep : C_ {
  const float* dgh; const float* whhT; const float* dhz;
  const float* masks; const int64_t* mask_idx;
  float* carry; int M, H;
  using ACtx = typename C_::ACtx;
  using BCtx = typename C_::BCtx;
  __device__ ACtx a_ctx(int m, int) const { return {dgh + (size_t)m * 3 * H, 0, 0, m < M}; }
  __device__ f32x4 a_load(const ACtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ BCtx b_ctx(int n, int) const { return {whhT + (size_t)n * 3 * H, 0, n < H}; }
  __device__ f32x4 b_load(const BCtx& c, int k) const {
    return c.ok ? *reinterpret_cast<const f32x4*>(c.p + k) : zero4();
  }
  __device__ void k_range(int, int& b, int& e) const { b = 0; e = 3 * H; }
  __device__ void store(int m, int n, int, float v) const {
    if (m >= M || n >= H) return;
    const float mk = masks ? masks[mask_idx ? mask_idx[m] : m] : 1.0f;
    const size_t o = (size_t)m * H + n;
    carry[o] = (v + dhz[o]) * mk;
  }
};

// gate gradients of one step: dh' = dout + carry;
//   dn = dh'(1-z), dz = dh'(h_in - n), da_n = dn(1-n²), dr = da_n·ghn,
//   da_r = dr·r(1-r), da_z = dz·z(1-z);  dgi = [da_r, da_z, da_n],
//   dgh = [da_r, da_z, da_n·r];  dhz = dh'·z
// (dgh·W_hh + dh'·z)·m(t), rounded as written
__device__ __forceinline__ float gru_carry(float v, float dhz, float m) {
#pragma clang fp contract(off)
  return (v + dhz) * m;
}

// explicitly rounded (no FMA contraction): the same bits in every kernel that
// inlines it (step launches, fused step + cell, persistent BPTT)
struct GruCellGrad {
  float dar, daz, dan, dghn, dhz;
};
__device__ __forceinline__ GruCellGrad gru_cell_grad(float dh, float rr, float zz, float nn, float ghn, float hin) {
#pragma clang fp contract(off)
  // plain operators under the pragma (HIP's __fmul_rn & co. are plain operators
  // compiled outside it, so they would still contract)
  const float dn = dh * (1.0f - zz);
  const float dz = dh * (hin - nn);
  const float dan = dn * (1.0f - nn * nn);
  const float dr = dan * ghn;
  const float dar = dr * rr * (1.0f - rr);
  const float daz = dz * zz * (1.0f - zz);
  return {dar, daz, dan, dan * rr, dh * zz};
}
__device__ __forceinline__ void gru_cell_bwd_elem(float dh, float rr, float zz, float nn, float ghn, float hin,
                                                  size_t i, size_t g, int H, float* __restrict__ dgi,
                                                  float* __restrict__ dgh, float* __restrict__ dhz) {
  const GruCellGrad c = gru_cell_grad(dh, rr, zz, nn, ghn, hin);
  dgi[g] = c.dar;
  dgi[g + H] = c.daz;
  dgi[g + 2 * H] = c.dan;
  dgh[g] = c.dar;
  dgh[g + H] = c.daz;
  dgh[g + 2 * H] = c.dghn;
  dhz[i] = c.dhz;
}

__global__ __launch_bounds__(256) void gru_cell_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ carry,
                                                           const float* __restrict__ r, const float* __restrict__ z,
                                                           const float* __restrict__ n, const float* __restrict__ ghn,
                                                           const float* __restrict__ hin, float* __restrict__ dgi,
                                                           float* __restrict__ dgh, float* __restrict__ dhz, int M,
                                                           int H, int has_carry) {
  const long long total = (long long)M * H;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int m = (int)(i / H), j = (int)(i - (long long)m * H);
    const float dh = dout[i] + (has_carry ? carry[i] : 0.f);
    gru_cell_bwd_elem(dh, r[i], z[i], n[i], ghn[i], hin[i], (size_t)i, (size_t)m * 3 * H + j, H, dgi, dgh, dhz);
  }
}

// W_ih [3H][I] -> W_ih padded [3H][Ip] (zeros), W_ihᵀ[:H] [H][3H], W_hhᵀ [H][3H]
__global__ __launch_bounds__(256) void gru_pack_kernel(const float* __restrict__ wih, const float* __restrict__ whh,
                                                       int H, int I, int Ip, float* __restrict__ wih_pad,
                                                       float* __restrict__ wihT, float* __restrict__ whhT) {
  const long long n0 = 3LL * H * Ip, n1 = (long long)H * 3 * H, n2 = n1;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n0 + n1 + n2; i += (long long)gridDim.x * 256) {
    long long q = i;
    if (q < n0) {
      const int g = (int)(q / Ip), k = (int)(q % Ip);
      wih_pad[q] = k < I ? wih[(size_t)g * I + k] : 0.f;
    } else if ((q -= n0) < n1) {
      const int j = (int)(q / (3 * H)), g = (int)(q % (3 * H));
      wihT[q] = wih[(size_t)g * I + j];
    } else {
      q -= n1;
      const int j = (int)(q / (3 * H)), g = (int)(q % (3 * H));
      whhT[q] = whh[(size_t)g * H + j];
    }
  }
}

// dst[r*ld + col0 + c] = src[row(r)*ncols + c] (c < ncols), zeros for ncols <= c < zero_to
__global__ __launch_bounds__(256) void concat_cols_kernel(const float* __restrict__ src, const int64_t* __restrict__ idx,
                                                          long long rows, int ncols, float* __restrict__ dst, int ld,
                                                          int col0, int zero_to) {
  const long long total = rows * zero_to;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i / zero_to;
    const int c = (int)(i - r * zero_to);
    const long long sr = idx ? idx[r] : r;
    dst[r * ld + col0 + c] = c < ncols ? src[sr * ncols + c] : 0.f;
  }
}

// idx[t*n + j] = t*N + envs[j]  (recurrent_generator sample order, storage.py:195-220)
__global__ __launch_bounds__(256) void rec_indices_kernel(const int64_t* __restrict__ envs, int n, int T, int N,
                                                          int64_t* __restrict__ idx) {
  const long long total = (long long)T * n;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int t = (int)(i / n), j = (int)(i - (long long)t * n);
    idx[i] = (int64_t)t * N + envs[j];
  }
}

using CfgGru = Cfg<32, 96, 1, 1, true, true>;     // one wave: 32 rows x (r,z,n) x 32 units
using CfgGruB = Cfg<64, 64, 2, 2, true, true>;

// ---------------------------------------------------------------------------
// Register-tiled step kernels.  A minibatch step has only n_env = 512 rows, so
// the tile GEMM above fills 128 waves (half the chip, one wave per CU) and each
// step is latency-bound (~40 us).  Here a block of 4 waves owns 32 rows x 16
// hidden units and splits K four ways; every operand goes global -> registers
// once per launch (no LDS staging, no k-loop barrier), one
// v_mfma_f32_16x16x4_f32 (exact fp32) per 16x16 tile per k-step, and the four
// K-quarter partials meet in LDS for the fused epilogue.  512 rows x 256 units
// -> 256 blocks.  K order: wave q owns the 4*KW consecutive k from q*4*KW, dealt
// to its lane groups in 16-B chunks — MFMA s of lane group g takes
// k = q*4*KW + 16*(s/4) + 4*g + s%4, the same k for the A and B operands — so one
// 16-B load instruction of the four lane groups reads 64 contiguous bytes of a
// row (one request; with KW-long runs per lane group it touched four 64-B
// segments per instruction, and the sc1 hand-off loads, which skip L1, re-fetched
// each segment four times).
// MFMA maps (16x16x4 f32): A[l&15][k=l>>4], B[k=l>>4][l&15], D col=l&15, row=4(l>>4)+r.

// forward: gh = h_in · W_hhᵀ for the (r, z, n) rows of the block's 16 units, then
// the GRU cell (as GruStep::store_tile).  The block's W_hh slice (b) is loaded by
// the caller: once per launch (step kernel) or once per sequence (persistent).
// PUB (persistent kernel): h is handed between blocks inside the launch — its
// stores are write-through (sc1) and every load of h is an sc1 load (the R1 form
// of cdna_hip_programming.md §6 G16: no release / acquire fence needed)
template <int H, bool PUB = false>
__device__ __forceinline__ void gru_fwd_tile(int m0, int j0, const float* __restrict__ hprev,
                                             const float* __restrict__ masks, const int64_t* __restrict__ mask_idx,
                                             const GruRow<H / 16, (H / 16) % 8 == 0> (&b)[3], const float* __restrict__ bhh,
                                             const float* __restrict__ gi, int M, float* __restrict__ hout,
                                             float* __restrict__ sr, float* __restrict__ sz, float* __restrict__ sn,
                                             float* __restrict__ sghn, float* __restrict__ shin,
                                             f32x4 (&P)[4][6][64]) {
  constexpr int KW = H / 16;   // k per lane group and wave (4 groups x 4 waves x KW = H)
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6, c = lane & 15, g = lane >> 4;
  const int kg = q * 4 * KW + 4 * g;   // + 4 s: the lane group's 16-B chunk of MFMAs s .. s + 3
  float a[2][KW];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int m = m0 + 16 * rt + c;
    const bool ok = m < M;
    const float mk = ok && masks ? masks[mask_idx ? mask_idx[m] : m] : 1.0f;
    const float* src = hprev + (size_t)(ok ? m : 0) * H + kg;
#pragma unroll
    for (int s = 0; s < KW; s += 4) {
      f32x4 v;
      if constexpr (PUB)
        v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                          make_rsrc(hprev, (uint32_t)M * H * 4), ((ok ? m : 0) * H + kg + 4 * s) * 4, 0, 16));
      else
        v = *reinterpret_cast<const f32x4*>(src + 4 * s);
      v = ok ? v * mk : zero4();
      a[rt][s] = v[0]; a[rt][s + 1] = v[1]; a[rt][s + 2] = v[2]; a[rt][s + 3] = v[3];
    }
  }
  // the epilogue's operands (gi, bias, mask, h) are loaded here, in flight during
  // the MFMAs, instead of a second dependent round trip after the K-quarter sum
  float pg[2][3], pb[2][3], pm[2], ph[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = tid + 256 * e, m = min(m0 + (p >> 4), M - 1), j = j0 + (p & 15);
    const float* gr = gi + (size_t)m * 3 * H;
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) {
      pg[e][gt] = gr[gt * H + j];
      pb[e][gt] = bhh[gt * H + j];
    }
    pm[e] = masks ? masks[mask_idx ? mask_idx[m] : m] : 1.0f;
    if constexpr (PUB)
      ph[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(make_rsrc(hprev, (uint32_t)M * H * 4),
                                                                             (m * H + j) * 4, 0, 16));
    else
      ph[e] = hprev[(size_t)m * H + j];
  }
  f32x4 acc[2][3];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) acc[rt][gt] = zero4();
  gru_mma<KW, 0>(a, b, acc);
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) P[q][rt * 3 + gt][lane] = acc[rt][gt];
  __syncthreads();
  // epilogue: thread -> (row, unit) pairs; the K quarters summed in a fixed order
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = tid + 256 * e, ml = p >> 4, jl = p & 15, m = m0 + ml, j = j0 + jl;
    if (m >= M) continue;
    const int rt = ml >> 4, ir = ml & 15, ln = jl + 16 * (ir >> 2), rg = ir & 3;
    float v[3];
#pragma unroll
    for (int gt = 0; gt < 3; ++gt)
      v[gt] = ((P[0][rt * 3 + gt][ln][rg] + P[1][rt * 3 + gt][ln][rg]) + P[2][rt * 3 + gt][ln][rg]) +
              P[3][rt * 3 + gt][ln][rg];
    const float ghr = v[0] + pb[e][0], ghz = v[1] + pb[e][1], ghn = v[2] + pb[e][2];
    const float r = sigm(pg[e][0] + ghr);
    const float z = sigm(pg[e][1] + ghz);
    const float n = tanhf(pg[e][2] + r * ghn);
    const float hin = ph[e] * pm[e];
    const size_t o = (size_t)m * H + j;
    const float hv = __fmaf_rn(z, hin, (1.0f - z) * n);   // explicit: same rounding in every instantiation
    if constexpr (PUB)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, hv), make_rsrc(hout, (uint32_t)M * H * 4),
                                            (int)o * 4, 0, 16);
    else
      hout[o] = hv;
    if (sr) {
      sr[o] = r;
      sz[o] = z;
      sn[o] = n;
      sghn[o] = ghn;
      shin[o] = hin;
    }
  }
}

template <int H>
__device__ __forceinline__ void gru_load_whh(const float* __restrict__ whh, int j0,
                                             GruRow<H / 16, (H / 16) % 8 == 0> (&b)[3]) {
  constexpr int KW = H / 16;
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6, c = lane & 15, g = lane >> 4;
  const int kg = q * 4 * KW + 4 * g;   // gru_fwd_tile's K order
#pragma unroll
  for (int gt = 0; gt < 3; ++gt) {
    const float* src = whh + ((size_t)gt * H + j0 + c) * H + kg;
    float v[KW];
#pragma unroll
    for (int s = 0; s < KW; s += 4) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(src + 4 * s);
      v[s] = x[0]; v[s + 1] = x[1]; v[s + 2] = x[2]; v[s + 3] = x[3];
    }
    gru_row_set(v, b[gt]);
  }
}

template <int H>
__global__ __launch_bounds__(256) void gru_step16_kernel(const float* __restrict__ hprev,
                                                         const float* __restrict__ masks,
                                                         const int64_t* __restrict__ mask_idx,
                                                         const float* __restrict__ whh, const float* __restrict__ bhh,
                                                         const float* __restrict__ gi, int M, float* __restrict__ hout,
                                                         float* __restrict__ sr, float* __restrict__ sz,
                                                         float* __restrict__ sn, float* __restrict__ sghn,
                                                         float* __restrict__ shin) {
  __shared__ f32x4 P[4][6][64];
  GruRow<H / 16, (H / 16) % 8 == 0> b[3];
  gru_load_whh<H>(whh, blockIdx.y * 16, b);
  // row groups blockIdx.x, + gridDim.x, ...: the W_hh slice (loaded and split once)
  // serves several groups where the rows outnumber the CUs (the rollout's 4,096)
  for (int x = blockIdx.x; 32 * x < M; x += gridDim.x) {
    gru_fwd_tile<H>(32 * x, blockIdx.y * 16, hprev, masks, mask_idx, b, bhh, gi, M, hout, sr, sz, sn, sghn, shin, P);
    __syncthreads();   // every wave has read P before the next group rewrites it
  }
}

// Persistent whole-sequence forward: the step kernel's blocks stay resident for
// all T steps, each with its W_hh slice in registers (loaded once).  Step t of row
// group x needs h(t-1) of its 32 rows from all H/16 unit blocks of the group, so
// the groups synchronise separately (no grid-wide barrier): a block publishes its
// h(t) tile (write-through sc1 stores drained by every wave, then one relaxed
// agent-scope counter increment of its group) and waits for the group's count
// before step t + 1 (relaxed polls), reading h only with sc1 loads — the R1
// hand-off of cdna_hip_programming.md §6 G16, correct wherever the blocks run.
// Co-residency: the grid (<= one block per CU) is resident by its size when the
// device is not shared; it is NOT guaranteed when another process's kernels hold
// CUs.  So every wait is bounded (spin_max polls) and fail-safe: a block whose
// wait runs out sets *err and returns at once, and every waiting block also polls
// *err and leaves as soon as it is set — no block computes with a stale h(t-1),
// and the error reaches the host after at most one bounded wait.  *err is sticky
// (the caller clears it): a launch that starts with it set returns immediately,
// and ppo_clip_adam_guarded skips the optimizer step while it is set, so a timed
// out minibatch never changes the parameters.
// The h-independent operands of step t + 1 (the A-row and epilogue masks, gi) are
// loaded during step t, after its publish — they are in flight while the block
// waits for its group — and the minibatch index rows two steps ahead, so no
// index -> mask chain sits on the per-step path; the biases are loaded once.
template <int H>
__global__ __launch_bounds__(256) void gru_seq16_kernel(const float* __restrict__ h0, const float* __restrict__ masks,
                                                        const int64_t* __restrict__ idx, const float* __restrict__ whh,
                                                        const float* __restrict__ bhh, const float* __restrict__ gi,
                                                        int T, int n, float* __restrict__ hout, float* __restrict__ sr,
                                                        float* __restrict__ sz, float* __restrict__ sn,
                                                        float* __restrict__ sghn, float* __restrict__ shin,
                                                        int* __restrict__ cnt, int* __restrict__ err, int spin_max) {
  constexpr int KW = H / 16;   // k per lane group and wave (as gru_fwd_tile)
  __shared__ f32x4 P[4][6][64];
  __shared__ int s_abort;
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6, c = lane & 15, g = lane >> 4;
  const int j0 = blockIdx.y * 16, m0 = blockIdx.x * 32, grp = blockIdx.x, need = H / 16;
  const int kg = q * 4 * KW + 4 * g;   // gru_fwd_tile's K order
  if (threadIdx.x == 0) s_abort = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_abort) return;   // an earlier launch on these words timed out: its outputs (and ours) are invalid
  GruRow<KW, KW % 8 == 0> b[3];
  gru_load_whh<H>(whh, j0, b);
  const bool sv = sr != nullptr;
  const auto rh = make_rsrc(hout, (uint32_t)((size_t)T * n * H * 4 < 0xffffffffu ? (size_t)T * n * H * 4 : 0xffffffffu));
  // rows this thread touches: A rows ra[rt] (row tile rt, lane c), epilogue rows re[e]
  int ra[2], re[2];
  bool oka[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int m = m0 + 16 * rt + c;
    oka[rt] = m < n;
    ra[rt] = oka[rt] ? m : 0;
  }
  float pb[2][3];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = tid + 256 * e;
    re[e] = min(m0 + (p >> 4), n - 1);
#pragma unroll
    for (int gt = 0; gt < 3; ++gt) pb[e][gt] = bhh[gt * H + j0 + (p & 15)];
  }
  // step operands: mask-plane offsets (through idx) two steps ahead, masks / gi one ahead
  long long xa[2][2], xe[2][2];   // [slot][r]: mask-plane index of step (slot parity)
  auto load_idx = [&](int t, int slot) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      xa[slot][r] = idx ? (long long)idx[(size_t)t * n + ra[r]] : (long long)t * n + ra[r];
      xe[slot][r] = idx ? (long long)idx[(size_t)t * n + re[r]] : (long long)t * n + re[r];
    }
  };
  float mA[2], pm[2], pg[2][3];
  auto load_step = [&](int t, int slot) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) mA[rt] = oka[rt] && masks ? masks[xa[slot][rt]] : 1.0f;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      pm[e] = masks ? masks[xe[slot][e]] : 1.0f;
      const float* gr = gi + ((size_t)t * n + re[e]) * 3 * H + j0 + ((tid + 256 * e) & 15);
#pragma unroll
      for (int gt = 0; gt < 3; ++gt) pg[e][gt] = gr[gt * H];
    }
  };
  if (masks) {
    load_idx(0, 0);
    if (T > 1) load_idx(1, 1);
  }
  load_step(0, 0);
  for (int t = 0; t < T; ++t) {
    const size_t o = (size_t)t * n * H;
    if (t > 0) {   // h(t-1) of the group's rows complete (all its unit blocks published)
      if (threadIdx.x == 0) {
        const int target = need * t;
        int it = 0, ab = 0;
        // spin bound 0: every wait gives up at once (the forced-timeout test mode)
        while (spin_max == 0 || __hip_atomic_load(cnt + grp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {   // another block gave up
            ab = 1;
            break;
          }
          if (++it > spin_max) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ab = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        s_abort = ab;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: h loads stay below the poll
      __syncthreads();
      if (s_abort) return;   // never compute step t from an incomplete h(t-1)
    }
    // h(t-1): the A operand (masked, as gru_fwd_tile) and the epilogue's h
    float a[2][KW], ph[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int s = 0; s < KW; s += 4) {
        f32x4 v;
        if (t == 0)
          v = *reinterpret_cast<const f32x4*>(h0 + (size_t)ra[rt] * H + kg + 4 * s);
        else
          v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rh, (int)((o - (size_t)n * H) + (size_t)ra[rt] * H + kg + 4 * s) * 4, 0, 16));
        v = oka[rt] ? v * mA[rt] : zero4();
        a[rt][s] = v[0]; a[rt][s + 1] = v[1]; a[rt][s + 2] = v[2]; a[rt][s + 3] = v[3];
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = j0 + ((tid + 256 * e) & 15);
      ph[e] = t == 0 ? h0[(size_t)re[e] * H + j]
                     : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     rh, (int)((o - (size_t)n * H) + (size_t)re[e] * H + j) * 4, 0, 16));
    }
    f32x4 acc[2][3];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int gt = 0; gt < 3; ++gt) acc[rt][gt] = zero4();
    gru_mma<KW, 0>(a, b, acc);   // gru_fwd_tile's products and order
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int gt = 0; gt < 3; ++gt) P[q][rt * 3 + gt][lane] = acc[rt][gt];
    __syncthreads();
    // epilogue (gru_fwd_tile's): the K quarters summed in a fixed order, the cell;
    // h stored first, the saved gates after the publish (no other block reads them)
    float keep[2][5];
    size_t ko[2];
    bool kv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      kv[e] = false;
      const int p = tid + 256 * e, ml = p >> 4, jl = p & 15, m = m0 + ml, j = j0 + jl;
      if (m >= n) continue;
      const int rt = ml >> 4, ir = ml & 15, ln = jl + 16 * (ir >> 2), rg = ir & 3;
      float v[3];
#pragma unroll
      for (int gt = 0; gt < 3; ++gt)
        v[gt] = ((P[0][rt * 3 + gt][ln][rg] + P[1][rt * 3 + gt][ln][rg]) + P[2][rt * 3 + gt][ln][rg]) +
                P[3][rt * 3 + gt][ln][rg];
      const float ghr = v[0] + pb[e][0], ghz = v[1] + pb[e][1], ghn = v[2] + pb[e][2];
      const float r = sigm(pg[e][0] + ghr);
      const float z = sigm(pg[e][1] + ghz);
      const float nn = tanhf(pg[e][2] + r * ghn);
      const float hin = ph[e] * pm[e];
      const size_t oo = o + (size_t)m * H + j;
      const float hv = __fmaf_rn(z, hin, (1.0f - z) * nn);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, hv), rh, (int)oo * 4, 0, 16);
      kv[e] = true;
      ko[e] = oo;
      keep[e][0] = r; keep[e][1] = z; keep[e][2] = nn; keep[e][3] = ghn; keep[e][4] = hin;
    }
    auto store_saves = [&]() {
      if (!sv) return;
#pragma unroll
      for (int e = 0; e < 2; ++e)
        if (kv[e]) {
          sr[ko[e]] = keep[e][0];
          sz[ko[e]] = keep[e][1];
          sn[ko[e]] = keep[e][2];
          sghn[ko[e]] = keep[e][3];
          shin[ko[e]] = keep[e][4];
        }
    };
    if (t + 1 < T) {   // publish h(t) of this tile
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its sc1 h stores done
      __syncthreads();   // also: every wave has read P before the next step rewrites it
      if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      store_saves();   // written during the wait
      // step t + 1's h-independent operands (in flight during the wait), t + 2's index rows
      load_step(t + 1, (t + 1) & 1);
      if (masks && t + 2 < T) load_idx(t + 2, t & 1);
    } else {
      store_saves();
    }
  }
}

// step t-1's cell-backward inputs/outputs, fused into step t's carry epilogue
// (dout NULL: no fusion).  dhz is read for step t and rewritten for t-1 by the
// same thread, element by element.
struct CellPrev {
  const float *dout, *r, *z, *n, *ghn, *hin;
  float *dgi, *dgh;
};

// backward: carry = (dgh · W_hh + dh'·z) · m(t) for the block's 32 rows x 16 units
// (B = W_hhᵀ packed [H][3H]: unit j's column of W_hh is row j, contiguous)
template <int H>
__global__ __launch_bounds__(256) void gru_step_bwd16_kernel(const float* __restrict__ dgh,
                                                             const float* __restrict__ whhT,
                                                             const float* __restrict__ dhz,
                                                             const float* __restrict__ masks,
                                                             const int64_t* __restrict__ mask_idx,
                                                             float* __restrict__ carry, int M,
                                                             const CellPrev cp) {
  constexpr int KW = 3 * H / 16;
  constexpr int NH = KW % 16 == 0 ? 2 : 1, KH = KW / NH;   // K halves keep the operand registers small
  constexpr bool BF = KH % 8 == 0;                         // split-bf16 products (gru_mma)
  __shared__ f32x4 P[4][2][64];
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6, c = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 32, j0 = blockIdx.y * 16;
  const int kg = q * 4 * KW + 4 * g;   // + half * 4 * KH + 4 s (gru_fwd_tile's chunked K order)
  // epilogue operands prefetched (in flight during the MFMAs)
  float pd[2], pm[2], pc[2][6];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = tid + 256 * e, m = min(m0 + (p >> 4), M - 1), j = j0 + (p & 15);
    const size_t o = (size_t)m * H + j;
    pd[e] = dhz[o];
    pm[e] = masks ? masks[mask_idx ? mask_idx[m] : m] : 1.0f;
    if (cp.dout) {
      pc[e][0] = cp.dout[o]; pc[e][1] = cp.r[o]; pc[e][2] = cp.z[o];
      pc[e][3] = cp.n[o]; pc[e][4] = cp.ghn[o]; pc[e][5] = cp.hin[o];
    }
  }
  f32x4 acc[2][1] = {{zero4()}, {zero4()}};
#pragma unroll
  for (int half = 0; half < NH; ++half) {
    float a[2][KH], b[KH];
    const int kb = kg + half * 4 * KH;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int m = m0 + 16 * rt + c;
      const bool ok = m < M;
      const float* src = dgh + (size_t)(ok ? m : 0) * 3 * H + kb;
#pragma unroll
      for (int s = 0; s < KH; s += 4) {
        const f32x4 v = ok ? *reinterpret_cast<const f32x4*>(src + 4 * s) : zero4();
        a[rt][s] = v[0]; a[rt][s + 1] = v[1]; a[rt][s + 2] = v[2]; a[rt][s + 3] = v[3];
      }
    }
    const float* bs = whhT + (size_t)(j0 + c) * 3 * H + kb;
#pragma unroll
    for (int s = 0; s < KH; s += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(bs + 4 * s);
      b[s] = v[0]; b[s + 1] = v[1]; b[s + 2] = v[2]; b[s + 3] = v[3];
    }
    GruRow<KH, BF> w[1];
    gru_row_set(b, w[0]);
    gru_mma<KH, 0>(a, w, acc);
  }
  P[q][0][lane] = acc[0][0];
  P[q][1][lane] = acc[1][0];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = tid + 256 * e, ml = p >> 4, jl = p & 15, m = m0 + ml, j = j0 + jl;
    if (m >= M) continue;
    const int rt = ml >> 4, ir = ml & 15, ln = jl + 16 * (ir >> 2), rg = ir & 3;
    const float v = ((P[0][rt][ln][rg] + P[1][rt][ln][rg]) + P[2][rt][ln][rg]) + P[3][rt][ln][rg];
    const size_t o = (size_t)m * H + j;
    const float cv = gru_carry(v, pd[e], pm[e]);
    carry[o] = cv;
    if (cp.dout)   // the previous step's cell backward for this element (gru_cell_bwd_kernel, fused)
      gru_cell_bwd_elem(pc[e][0] + cv, pc[e][1], pc[e][2], pc[e][3], pc[e][4], pc[e][5], o,
                        (size_t)m * 3 * H + j, H, cp.dgi, cp.dgh, const_cast<float*>(dhz));
  }
}

// Persistent backward through time (model.py:116-165 reversed): the blocks of
// gru_step_bwd16_kernel stay resident for steps T-1 .. 1, each with its W_hhᵀ
// slice in registers (loaded once).  Step t of row group x needs dgh(t) of its 32
// rows over all 3H columns, written by all H/16 unit blocks of the group in the
// previous iteration (the cell backward of step t fused into step t+1's epilogue;
// step T-1's by the ppo_gru_cell_bwd launch before this kernel): the same R1
// hand-off as gru_seq16_kernel — dgh(t-1) stored write-through (sc1), drained,
// one relaxed counter increment of the group; dgh loaded with sc1 loads; bounded,
// fail-safe waits on the shared error word.  The per-element arithmetic, the
// K-quarter / K-half order and the MFMA sequence are those of the step kernel, so
// the results equal the T - 1 step launches bit for bit.
template <int H>
__global__ __launch_bounds__(256) void gru_seq_bwd16_kernel(
    const float* __restrict__ dout, const float* __restrict__ sr, const float* __restrict__ sz,
    const float* __restrict__ sn, const float* __restrict__ sghn, const float* __restrict__ shin,
    const float* __restrict__ masks, const int64_t* __restrict__ idx, const float* __restrict__ whhT, int T, int n,
    float* __restrict__ dgi, float* __restrict__ dgh, float* __restrict__ dhz, float* __restrict__ carry,
    int* __restrict__ cnt, int* __restrict__ err, int spin_max) {
  constexpr int KW = 3 * H / 16;
  constexpr int NH = KW % 16 == 0 ? 2 : 1, KH = KW / NH;
  constexpr bool BF = KH % 8 == 0;
  __shared__ f32x4 P[4][2][64];
  __shared__ int s_abort;
  const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6, c = lane & 15, g = lane >> 4;
  const int grp = blockIdx.x, m0 = grp * 32, j0 = blockIdx.y * 16, need = H / 16;
  const int kg = q * 4 * KW + 4 * g;   // gru_step_bwd16_kernel's K order
  if (tid == 0) s_abort = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_abort) return;
  GruRow<KW, BF> w[1];   // W_hhᵀ row j0 + c: value half * KH + s at k = kg + half * 4 KH + 4 s (+ 0..3)
  {
    float b[KW];
    const float* bs = whhT + (size_t)(j0 + c) * 3 * H + kg;
#pragma unroll
    for (int half = 0; half < NH; ++half)
#pragma unroll
      for (int s = 0; s < KH; s += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(bs + half * 4 * KH + 4 * s);
        b[half * KH + s] = v[0]; b[half * KH + s + 1] = v[1]; b[half * KH + s + 2] = v[2]; b[half * KH + s + 3] = v[3];
      }
    gru_row_set(b, w[0]);
  }
  // dgh hand-off (MI355X_MICROARCH "Correctness boundaries", hand-off table row 1):
  // every dgh store is write-through (sc1), each storing wave drains (vmcnt(0)) and
  // joins a barrier before lane 0 adds to the group counter (relaxed, agent scope);
  // the consumer polls the counter, joins a barrier, then loads dgh with sc1 (the
  // CU's L1 bypassed).  Round 6: the L2 variant (plain stores
  // where a row group's unit blocks shared one XCD, checked by their XCC_IDs) bought
  // 1.8 % of gru_seq_bwd at c5 (1.972-1.992 vs 2.011-2.019 ms, same box, alternating,
  // profiles/r06_c_l2ab.log) for a form outside the guide's table, and was removed.
  // Block (x, 0) reports that its group ran persistent (1) in the counter buffer.
  if (tid == 0 && blockIdx.y == 0)
    __hip_atomic_store(cnt + gridDim.x + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t gbytes = (uint32_t)((size_t)n * 3 * H * 4);
  // the epilogue's elements (as gru_step_bwd16_kernel): rows re[e] (clamped), units je[e]
  int re[2], je[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int p = tid + 256 * e;
    re[e] = min(m0 + (p >> 4), n - 1);
    je[e] = j0 + (p & 15);
  }
  // h-independent operands of step t - 1 (its mask, the saved activations of step
  // t - 2) loaded during step t after its publish, the index rows two steps ahead;
  // dhz carried in registers (the thread wrote it in the step before)
  long long xe[2][2];
  auto load_idx = [&](int t, int slot) {
#pragma unroll
    for (int e = 0; e < 2; ++e) xe[slot][e] = idx ? (long long)idx[(size_t)t * n + re[e]] : (long long)t * n + re[e];
  };
  float pd[2], pm[2], pc[2][6];
  auto load_step = [&](int t, int slot) {
    const size_t op = (size_t)(t - 1) * n * H;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const size_t oe = (size_t)re[e] * H + je[e];
      pm[e] = masks ? masks[xe[slot][e]] : 1.0f;
      pc[e][0] = dout[op + oe]; pc[e][1] = sr[op + oe]; pc[e][2] = sz[op + oe];
      pc[e][3] = sn[op + oe]; pc[e][4] = sghn[op + oe]; pc[e][5] = shin[op + oe];
    }
  };
  if (masks) {
    load_idx(T - 1, (T - 1) & 1);
    if (T - 2 >= 1) load_idx(T - 2, (T - 2) & 1);
  }
  load_step(T - 1, (T - 1) & 1);
#pragma unroll
  for (int e = 0; e < 2; ++e) pd[e] = dhz[(size_t)re[e] * H + je[e]];
  constexpr int CP_ST = 16, CP_LD = 16;   // sc1 stores and loads of dgh
  for (int t = T - 1; t >= 1; --t) {
    if (t < T - 1) {   // dgh(t) of the group's rows complete
      if (tid == 0) {
        const int target = need * (T - 1 - t);
        int it = 0, ab = 0;
        // spin bound 0: every wait gives up at once (the forced-timeout test mode)
        while (spin_max == 0 || __hip_atomic_load(cnt + grp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            ab = 1;
            break;
          }
          if (++it > spin_max) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ab = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        s_abort = ab;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: dgh loads stay below the poll
      __syncthreads();
      if (s_abort) return;
    }
    const size_t o = (size_t)t * n * H, op = o - (size_t)n * H;
    const auto rs = make_rsrc(dgh + 3 * o, gbytes);
    f32x4 acc[2][1] = {{zero4()}, {zero4()}};
#pragma unroll
    for (int half = 0; half < NH; ++half) {
      float a[2][KH];
      const int kb = kg + half * 4 * KH;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int m = m0 + 16 * rt + c;
        const bool ok = m < n;
#pragma unroll
        for (int s = 0; s < KH; s += 4) {
          f32x4 v = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ((ok ? m : 0) * 3 * H + kb + 4 * s) * 4, 0, CP_LD));
          v = ok ? v : zero4();
          a[rt][s] = v[0]; a[rt][s + 1] = v[1]; a[rt][s + 2] = v[2]; a[rt][s + 3] = v[3];
        }
      }
      if (half == 0) gru_mma<KH, 0>(a, w, acc);   // the step kernel's products and order
      else gru_mma<KH, KH>(a, w, acc);
    }
    P[q][0][lane] = acc[0][0];
    P[q][1][lane] = acc[1][0];
    __syncthreads();
    float* dgh_p = dgh + 3 * op;
    const auto rsp = make_rsrc(dgh_p, gbytes);
    // dgh stored first; dgi, carry and dhz after the publish (no other block reads them)
    float keep[2][5];
    size_t ko[2], kg[2];
    bool kv[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      kv[e] = false;
      const int p = tid + 256 * e, ml = p >> 4, jl = p & 15, m = m0 + ml, j = j0 + jl;
      if (m >= n) continue;
      const int rt = ml >> 4, ir = ml & 15, ln = jl + 16 * (ir >> 2), rg = ir & 3;
      const float v = ((P[0][rt][ln][rg] + P[1][rt][ln][rg]) + P[2][rt][ln][rg]) + P[3][rt][ln][rg];
      const size_t oe = (size_t)m * H + j;
      const float cv = gru_carry(v, pd[e], pm[e]);
      // gru_cell_bwd_elem for step t - 1, dgh stored write-through for the group
      const GruCellGrad cg = gru_cell_grad(pc[e][0] + cv, pc[e][1], pc[e][2], pc[e][3], pc[e][4], pc[e][5]);
      const size_t gg = (size_t)m * 3 * H + j;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, cg.dar), rsp, (int)gg * 4, 0, CP_ST);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, cg.daz), rsp, (int)(gg + H) * 4, 0, CP_ST);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, cg.dghn), rsp, (int)(gg + 2 * H) * 4, 0, CP_ST);
      kv[e] = true;
      ko[e] = oe;
      kg[e] = gg;
      keep[e][0] = cv; keep[e][1] = cg.dar; keep[e][2] = cg.daz; keep[e][3] = cg.dan; keep[e][4] = cg.dhz;
      pd[e] = cg.dhz;   // the next step's dhz operand
    }
    auto store_rest = [&]() {
      float* dgi_p = dgi + 3 * op;
#pragma unroll
      for (int e = 0; e < 2; ++e)
        if (kv[e]) {
          carry[ko[e]] = keep[e][0];
          dgi_p[kg[e]] = keep[e][1];
          dgi_p[kg[e] + H] = keep[e][2];
          dgi_p[kg[e] + 2 * H] = keep[e][3];
          dhz[ko[e]] = keep[e][4];
        }
    };
    if (t > 1) {   // publish dgh(t - 1) of this tile
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();   // also: every wave has read P before the next step rewrites it
      if (tid == 0) __hip_atomic_fetch_add(cnt + grp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      store_rest();   // written during the wait
      load_step(t - 1, (t - 1) & 1);   // in flight during the wait
      if (masks && t - 2 >= 1) load_idx(t - 2, t & 1);
    } else {
      store_rest();
    }
  }
}

// 0: register-tiled step kernels where H allows; 1: the tile-GEMM steps (A/B)
static int g_gru_variant = 0;
// persistent whole-sequence launches where the grid fits one block per CU, bit 0:
// forward (gru_seq16_kernel), bit 1: backward (gru_seq_bwd16_kernel); clear bits
// run one step kernel per step.  Both by default since each loads its next step's
// h-independent operands during the group wait (n = 512, H = 256: forward 7.1 vs
// 8.7 us per step launched, BPTT 10.0 vs 10.2; before that prefetch the persistent
// BPTT was the slower, 12.6 vs 10.9)
static int g_gru_persist = 3;

// bounded-wait length of the persistent kernels (polls of ~64 clocks each; 0: every
// wait times out, which the fail-safe tests use)
static int g_gru_spin = 1 << 21;

// Library-held synchronisation words for ppo_gru_seq_fwd (callers that pass their
// own use ppo_gru_seq_fwd_ws): one buffer {err, counters...} per (device, stream),
// so launches in flight on different streams or devices never share counters.
// Grow-only; a buffer is reallocated only after its stream has drained.
struct PersistWords {
  int dev;
  hipStream_t stream;
  int* buf;
  int cap;
};
static std::mutex g_words_mu;
static PersistWords g_words[64];
static int g_nwords = 0;

static int* persist_words(hipStream_t st, int groups) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_words_mu);
  PersistWords* w = nullptr;
  for (int i = 0; i < g_nwords; ++i)
    if (g_words[i].dev == dev && g_words[i].stream == st) w = &g_words[i];
  if (!w) {
    if (g_nwords == 64) return nullptr;
    w = &g_words[g_nwords++];
    *w = PersistWords{dev, st, nullptr, 0};
  }
  if (groups + 1 > w->cap) {
    if (w->buf) {
      if (hipStreamSynchronize(st) != hipSuccess) return nullptr;   // the old buffer's launches are done
      (void)hipFree(w->buf);
    }
    const int cap = groups + 1 > 4096 ? groups + 1 : 4096;
    w->buf = nullptr;
    w->cap = 0;
    if (hipMalloc(&w->buf, (size_t)cap * sizeof(int)) != hipSuccess) return (w->buf = nullptr);
    if (hipMemset(w->buf, 0, (size_t)cap * sizeof(int)) != hipSuccess) return nullptr;
    w->cap = cap;
  }
  return w->buf;
}

static int gru_cus() {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    n_cu = v;
  }
  return n_cu;
}

template <int H>
int launch_seq16(const float* h0, const float* masks, const int64_t* idx, const float* whh, const float* bhh,
                 const float* gi, int T, int n, float* hout, float* sr, float* sz, float* sn, float* sghn,
                 float* shin, int* cnt, int* err, hipStream_t st) {
  const int groups = ceil_div(n, 32);
  PPO_HIP_CHECK(hipMemsetAsync(cnt, 0, (size_t)groups * sizeof(int), st), "ppo_gru_seq_fwd: counter reset");
  dim3 grid((unsigned)groups, H / 16);
  gru_seq16_kernel<H><<<grid, 256, 0, st>>>(h0, masks, idx, whh, bhh, gi, T, n, hout, sr, sz, sn, sghn, shin, cnt, err,
                                            g_gru_spin);
  PPO_LAUNCH_CHECK("gru_seq16_kernel");
  return 0;
}

template <int H>
int launch_step16(const float* hprev, const float* masks, const int64_t* mask_idx, const float* whh,
                  const float* bhh, const float* gi, int M, float* hout, float* sr, float* sz, float* sn,
                  float* sghn, float* shin, hipStream_t st) {
  // at most two blocks per CU: more row groups than that loop inside a block
  const int n_cu = gru_cus();
  // (4,096 rows, H = 256: 0.030 -> 0.021 ms; one, three or four blocks per CU 0.024-0.028,
  // profiles/r05_n_gru_step.log)
  const int gx = std::min((int)ceil_div(M, 32), std::max(1, 2 * n_cu / (H / 16)));
  dim3 grid((unsigned)gx, H / 16);
  gru_step16_kernel<H><<<grid, 256, 0, st>>>(hprev, masks, mask_idx, whh, bhh, gi, M, hout, sr, sz, sn, sghn, shin);
  PPO_LAUNCH_CHECK("gru_step16_kernel");
  return 0;
}

template <int H>
int launch_step_bwd16(const float* dgh, const float* whhT, const float* dhz, const float* masks,
                      const int64_t* mask_idx, float* carry, int M, hipStream_t st, const CellPrev& cp = CellPrev{}) {
  dim3 grid((unsigned)ceil_div(M, 32), H / 16);
  gru_step_bwd16_kernel<H><<<grid, 256, 0, st>>>(dgh, whhT, dhz, masks, mask_idx, carry, M, cp);
  PPO_LAUNCH_CHECK("gru_step_bwd16_kernel");
  return 0;
}

template <int H>
int launch_seq_bwd16(const float* dout, const float* sr, const float* sz, const float* sn, const float* sghn,
                     const float* shin, const float* masks, const int64_t* idx, const float* whhT, int T, int n,
                     float* dgi, float* dgh, float* dhz, float* carry, int* cnt, int* err, hipStream_t st) {
  const int groups = ceil_div(n, 32);
  PPO_HIP_CHECK(hipMemsetAsync(cnt, 0, (size_t)groups * 2 * sizeof(int), st), "ppo_gru_seq_bwd: counter reset");
  dim3 grid((unsigned)groups, H / 16);
  gru_seq_bwd16_kernel<H><<<grid, 256, 0, st>>>(dout, sr, sz, sn, sghn, shin, masks, idx, whhT, T, n, dgi, dgh, dhz,
                                                carry, cnt, err, g_gru_spin);
  PPO_LAUNCH_CHECK("gru_seq_bwd16_kernel");
  return 0;
}

static unsigned grid_for(long long total) {
  long long b = (total + 255) / 256;
  return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace

// one GRU step, fused cell (model.py:112-115 single step, or one step of :116-165)
PPO_API int ppo_gru_step_fwd(const float* hprev, const float* masks, const int64_t* mask_idx, const float* whh,
                             const float* bhh, const float* gi, int M, int H, float* hout, float* save_r, float* save_z,
                             float* save_n, float* save_ghn, float* save_hin, void* stream) {
  PPO_REQUIRE(M >= 0 && H > 0 && H % 32 == 0, "ppo_gru_step_fwd: M=%d H=%d (H multiple of 32)", M, H);
  if (M == 0) return 0;
  if (g_gru_variant == 0) {
    hipStream_t st = as_stream(stream);
    switch (H) {
      case 64: return launch_step16<64>(hprev, masks, mask_idx, whh, bhh, gi, M, hout, save_r, save_z, save_n,
                                        save_ghn, save_hin, st);
      case 128: return launch_step16<128>(hprev, masks, mask_idx, whh, bhh, gi, M, hout, save_r, save_z, save_n,
                                          save_ghn, save_hin, st);
      case 256: return launch_step16<256>(hprev, masks, mask_idx, whh, bhh, gi, M, hout, save_r, save_z, save_n,
                                          save_ghn, save_hin, st);
      case 512: return launch_step16<512>(hprev, masks, mask_idx, whh, bhh, gi, M, hout, save_r, save_z, save_n,
                                          save_ghn, save_hin, st);
    }
  }
  GruStep<CfgGru> p;
  p.hprev = hprev; p.masks = masks; p.mask_idx = mask_idx; p.whh = whh; p.bhh = bhh; p.gi = gi; p.hout = hout;
  p.sr = save_r; p.sz = save_z; p.sn = save_n; p.sghn = save_ghn; p.shin = save_hin; p.M = M; p.H = H;
  return launch(p, M, 3 * H, 1, as_stream(stream), "gru_step_fwd", 2.0 * M * 3 * H * H);
}

PPO_API int ppo_gru_cell_bwd(const float* dout, const float* carry, const float* r, const float* z, const float* n,
                             const float* ghn, const float* hin, float* dgi, float* dgh, float* dhz, int M, int H,
                             int has_carry, void* stream) {
  PPO_REQUIRE(M >= 0 && H > 0, "ppo_gru_cell_bwd: M=%d H=%d", M, H);
  if (M == 0) return 0;
  gru_cell_bwd_kernel<<<grid_for((long long)M * H), 256, 0, as_stream(stream)>>>(dout, carry, r, z, n, ghn, hin, dgi,
                                                                                 dgh, dhz, M, H, has_carry);
  PPO_LAUNCH_CHECK("gru_cell_bwd_kernel");
  return 0;
}

PPO_API int ppo_gru_step_bwd(const float* dgh, const float* whhT, const float* dhz, const float* masks,
                             const int64_t* mask_idx, float* carry, int M, int H, void* stream) {
  PPO_REQUIRE(M >= 0 && H > 0 && H % 4 == 0, "ppo_gru_step_bwd: M=%d H=%d", M, H);
  if (M == 0) return 0;
  if (g_gru_variant == 0) {
    hipStream_t st = as_stream(stream);
    switch (H) {
      case 64: return launch_step_bwd16<64>(dgh, whhT, dhz, masks, mask_idx, carry, M, st);
      case 128: return launch_step_bwd16<128>(dgh, whhT, dhz, masks, mask_idx, carry, M, st);
      case 256: return launch_step_bwd16<256>(dgh, whhT, dhz, masks, mask_idx, carry, M, st);
      case 512: return launch_step_bwd16<512>(dgh, whhT, dhz, masks, mask_idx, carry, M, st);
    }
  }
  GruBwdStep<CfgGruB> p;
  p.dgh = dgh; p.whhT = whhT; p.dhz = dhz; p.masks = masks; p.mask_idx = mask_idx; p.carry = carry; p.M = M; p.H = H;
  return launch(p, M, H, 1, as_stream(stream), "gru_step_bwd", 2.0 * M * 3 * H * H);
}

// step t's carry GEMM fused with step t-1's cell backward (the BPTT loop body:
// ppo_gru_step_bwd(t) then ppo_gru_cell_bwd(t-1, carry) in one launch)
PPO_API int ppo_gru_step_bwd_cell(const float* dgh, const float* whhT, float* dhz, const float* masks,
                                  const int64_t* mask_idx, float* carry, int M, int H, const float* dout_prev,
                                  const float* r, const float* z, const float* n, const float* ghn, const float* hin,
                                  float* dgi_prev, float* dgh_prev, void* stream) {
  PPO_REQUIRE(M >= 0 && (H == 64 || H == 128 || H == 256 || H == 512) && g_gru_variant == 0,
              "ppo_gru_step_bwd_cell: M=%d H=%d (H in 64/128/256/512, register-tiled variant)", M, H);
  if (M == 0) return 0;
  const CellPrev cp{dout_prev, r, z, n, ghn, hin, dgi_prev, dgh_prev};
  hipStream_t st = as_stream(stream);
  switch (H) {
    case 64: return launch_step_bwd16<64>(dgh, whhT, dhz, masks, mask_idx, carry, M, st, cp);
    case 128: return launch_step_bwd16<128>(dgh, whhT, dhz, masks, mask_idx, carry, M, st, cp);
    case 256: return launch_step_bwd16<256>(dgh, whhT, dhz, masks, mask_idx, carry, M, st, cp);
    default: return launch_step_bwd16<512>(dgh, whhT, dhz, masks, mask_idx, carry, M, st, cp);
  }
}

PPO_API int ppo_gru_variant_get(void) { return g_gru_variant; }

// Whole-sequence loops (model.py:116-165 forward; its backward through time) run
// from C: one ABI call per minibatch instead of T (or 2T) Python->ctypes calls,
// which at ~10 us per step kernel were the critical path of the recurrent update.
// Rows of step t are t*n .. t*n + n - 1; mask of row j at step t: masks[idx[t*n + j]]
// (idx NULL: masks[t*n + j]).
// per 32-row group: the step counter, the BPTT's start counter, XCC_ID slots of up
// to 32 unit blocks (gru_seq_bwd16_kernel's L2 agreement) and the BPTT's path
// report; layout [G step counters][G start counters][32 G XCC slots][G paths]
// with G = ceil(n/32), path 1 = sc1 hand-off, 2 = L2 hand-off, 0 = not run
PPO_API int ppo_gru_seq_counters(int n) { return n > 0 ? ceil_div(n, 32) * 2 : 1; }

PPO_API int ppo_gru_seq_fwd_ws(const float* h0, const float* masks, const int64_t* idx, const float* whh,
                               const float* bhh, const float* gi, int T, int n, int H, float* hout, float* save_r,
                               float* save_z, float* save_n, float* save_ghn, float* save_hin, int* counters, int* err,
                               void* stream) {
  PPO_REQUIRE(T >= 0 && n >= 0 && H > 0 && H % 32 == 0, "ppo_gru_seq_fwd: T=%d n=%d H=%d", T, n, H);
  ProfScope prof("gru_seq_fwd", as_stream(stream), 2.0 * T * n * 3.0 * H * H);
  if (T > 0 && n > 0 && g_gru_variant == 0 && (g_gru_persist & 1) && (long long)ceil_div(n, 32) * (H / 16) <= gru_cus() &&
      (H == 64 || H == 128 || H == 256 || H == 512) && (long long)T * n * H * 4 < (1LL << 31)) {   // 32-bit offsets
    PPO_REQUIRE(counters != nullptr && err != nullptr, "ppo_gru_seq_fwd_ws: the persistent launch needs counters "
                                                       "(ppo_gru_seq_counters(n) ints) and an error word");
    hipStream_t st = as_stream(stream);
    switch (H) {
      case 64: return launch_seq16<64>(h0, masks, idx, whh, bhh, gi, T, n, hout, save_r, save_z, save_n, save_ghn, save_hin, counters, err, st);
      case 128: return launch_seq16<128>(h0, masks, idx, whh, bhh, gi, T, n, hout, save_r, save_z, save_n, save_ghn, save_hin, counters, err, st);
      case 256: return launch_seq16<256>(h0, masks, idx, whh, bhh, gi, T, n, hout, save_r, save_z, save_n, save_ghn, save_hin, counters, err, st);
      default: return launch_seq16<512>(h0, masks, idx, whh, bhh, gi, T, n, hout, save_r, save_z, save_n, save_ghn, save_hin, counters, err, st);
    }
  }
  const bool sv = save_r != nullptr;
  for (int t = 0; t < T; ++t) {
    const size_t o = (size_t)t * n * H;
    // with idx the mask plane is indexed through it; without, masks is [T][n]
    const float* mk = masks && !idx ? masks + (size_t)t * n : masks;
    const int rc = ppo_gru_step_fwd(t == 0 ? h0 : hout + o - (size_t)n * H, mk, idx ? idx + (size_t)t * n : nullptr,
                                    whh, bhh, gi + 3 * o, n, H, hout + o, sv ? save_r + o : nullptr,
                                    sv ? save_z + o : nullptr, sv ? save_n + o : nullptr, sv ? save_ghn + o : nullptr,
                                    sv ? save_hin + o : nullptr, stream);
    if (rc) return rc;
  }
  return 0;
}

// the same with the library's per-(device, stream) words (ppo_gru_persist_timeouts reads them)
PPO_API int ppo_gru_seq_fwd(const float* h0, const float* masks, const int64_t* idx, const float* whh,
                            const float* bhh, const float* gi, int T, int n, int H, float* hout, float* save_r,
                            float* save_z, float* save_n, float* save_ghn, float* save_hin, void* stream) {
  int* w = nullptr;
  if (T > 0 && n > 0 && (g_gru_persist & 1)) {
    w = persist_words(as_stream(stream), ppo_gru_seq_counters(n));
    PPO_REQUIRE(w != nullptr, "ppo_gru_seq_fwd: counter allocation failed");
  }
  return ppo_gru_seq_fwd_ws(h0, masks, idx, whh, bhh, gi, T, n, H, hout, save_r, save_z, save_n, save_ghn, save_hin,
                            w ? w + 1 : nullptr, w, stream);
}

PPO_API int ppo_gru_seq_bwd_ws(const float* dout, const float* save_r, const float* save_z, const float* save_n,
                               const float* save_ghn, const float* save_hin, const float* masks, const int64_t* idx,
                               const float* whhT, int T, int n, int H, float* dgi, float* dgh, float* dhz,
                               float* carry, int* counters, int* err, void* stream) {
  PPO_REQUIRE(T >= 0 && n >= 0 && H > 0 && H % 4 == 0, "ppo_gru_seq_bwd: T=%d n=%d H=%d", T, n, H);
  ProfScope prof("gru_seq_bwd", as_stream(stream), 2.0 * T * n * 3.0 * H * H);
  const bool fused = (H == 64 || H == 128 || H == 256 || H == 512) && g_gru_variant == 0;
  if (T > 1 && n > 0 && fused && (g_gru_persist & 2) && (long long)ceil_div(n, 32) * (H / 16) <= gru_cus()) {
    PPO_REQUIRE(counters != nullptr && err != nullptr, "ppo_gru_seq_bwd_ws: the persistent launch needs counters "
                                                       "(ppo_gru_seq_counters(n) ints) and an error word");
    const size_t o = (size_t)(T - 1) * n * H;   // step T - 1's cell backward (no carry), then steps T-1 .. 1
    int rc = ppo_gru_cell_bwd(dout + o, carry, save_r + o, save_z + o, save_n + o, save_ghn + o, save_hin + o,
                              dgi + 3 * o, dgh + 3 * o, dhz, n, H, 0, stream);
    if (rc) return rc;
    hipStream_t st = as_stream(stream);
    switch (H) {
      case 64: return launch_seq_bwd16<64>(dout, save_r, save_z, save_n, save_ghn, save_hin, masks, idx, whhT, T, n, dgi, dgh, dhz, carry, counters, err, st);
      case 128: return launch_seq_bwd16<128>(dout, save_r, save_z, save_n, save_ghn, save_hin, masks, idx, whhT, T, n, dgi, dgh, dhz, carry, counters, err, st);
      case 256: return launch_seq_bwd16<256>(dout, save_r, save_z, save_n, save_ghn, save_hin, masks, idx, whhT, T, n, dgi, dgh, dhz, carry, counters, err, st);
      default: return launch_seq_bwd16<512>(dout, save_r, save_z, save_n, save_ghn, save_hin, masks, idx, whhT, T, n, dgi, dgh, dhz, carry, counters, err, st);
    }
  }
  for (int t = T - 1; t >= 0; --t) {
    const size_t o = (size_t)t * n * H, op = o - (size_t)n * H;
    int rc = 0;
    if (!fused || t == T - 1)
      rc = ppo_gru_cell_bwd(dout + o, carry, save_r + o, save_z + o, save_n + o, save_ghn + o, save_hin + o,
                            dgi + 3 * o, dgh + 3 * o, dhz, n, H, t < T - 1, stream);
    if (!rc && t > 0) {
      const int64_t* mi = idx ? idx + (size_t)t * n : nullptr;
      const float* mk = masks && !idx ? masks + (size_t)t * n : masks;
      rc = fused ? ppo_gru_step_bwd_cell(dgh + 3 * o, whhT, dhz, mk, mi, carry, n, H, dout + op, save_r + op,
                                         save_z + op, save_n + op, save_ghn + op, save_hin + op, dgi + 3 * op,
                                         dgh + 3 * op, stream)
                 : ppo_gru_step_bwd(dgh + 3 * o, whhT, dhz, mk, mi, carry, n, H, stream);
    }
    if (rc) return rc;
  }
  return 0;
}

// the same with the library's per-(device, stream) words (ppo_gru_persist_timeouts reads them)
PPO_API int ppo_gru_seq_bwd(const float* dout, const float* save_r, const float* save_z, const float* save_n,
                            const float* save_ghn, const float* save_hin, const float* masks, const int64_t* idx,
                            const float* whhT, int T, int n, int H, float* dgi, float* dgh, float* dhz, float* carry,
                            void* stream) {
  int* w = nullptr;
  if (T > 1 && n > 0 && (g_gru_persist & 2)) {
    w = persist_words(as_stream(stream), ppo_gru_seq_counters(n));
    PPO_REQUIRE(w != nullptr, "ppo_gru_seq_bwd: counter allocation failed");
  }
  return ppo_gru_seq_bwd_ws(dout, save_r, save_z, save_n, save_ghn, save_hin, masks, idx, whhT, T, n, H, dgi, dgh, dhz,
                            carry, w ? w + 1 : nullptr, w, stream);
}

// persistent whole-sequence kernels on (1) / off (0)
PPO_API int ppo_gru_persist_set(int v) {
  PPO_REQUIRE(v >= 0 && v <= 3, "ppo_gru_persist_set: %d (bit 0 forward, bit 1 backward)", v);
  g_gru_persist = v;
  return 0;
}
PPO_API int ppo_gru_persist_get(void) { return g_gru_persist; }

// bounded-wait length (polls) of the persistent kernels; tests force a timeout with 1
PPO_API int ppo_gru_persist_spin_set(int polls) {
  PPO_REQUIRE(polls >= 0, "ppo_gru_persist_spin_set: %d", polls);
  g_gru_spin = polls;
  return 0;
}

// 1 if a ppo_gru_seq_fwd launch on `stream` timed out since the last call (its
// results are invalid), else 0; reads the library's word for (this device,
// stream) in stream order — waits for that stream only — and clears it
PPO_API int ppo_gru_persist_timeouts(void* stream) {
  hipStream_t st = as_stream(stream);
  int* w = persist_words(st, 0);
  if (w == nullptr) {
    ppo_set_error("ppo_gru_persist_timeouts: no counter buffer");
    return -1;
  }
  int v = 0;
  if (hipMemcpyAsync(&v, w, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    ppo_set_error("ppo_gru_persist_timeouts: read failed");
    return -1;
  }
  if (v && hipMemsetAsync(w, 0, sizeof(int), st) != hipSuccess) return -1;
  return v;
}

// A/B switch for the step kernels (0 register-tiled, 1 tile GEMM)
PPO_API int ppo_gru_variant_set(int v) {
  PPO_REQUIRE(v == 0 || v == 1, "ppo_gru_variant_set: %d", v);
  g_gru_variant = v;
  return 0;
}

PPO_API int ppo_gru_pack(const float* wih, const float* whh, int H, int I, int Ip, float* wih_pad, float* wihT,
                         float* whhT, void* stream) {
  PPO_REQUIRE(H > 0 && I > 0 && Ip >= I && Ip % 4 == 0, "ppo_gru_pack: H=%d I=%d Ip=%d", H, I, Ip);
  gru_pack_kernel<<<grid_for(3LL * H * Ip + 6LL * H * H), 256, 0, as_stream(stream)>>>(wih, whh, H, I, Ip, wih_pad,
                                                                                      wihT, whhT);
  PPO_LAUNCH_CHECK("gru_pack_kernel");
  return 0;
}

PPO_API int ppo_concat_cols(const float* src, const int64_t* idx, long long rows, int ncols, float* dst, int ld,
                            int col0, int zero_to, void* stream) {
  PPO_REQUIRE(rows >= 0 && ncols >= 0 && zero_to >= ncols && col0 + zero_to <= ld, "ppo_concat_cols: bad shape");
  if (rows == 0 || zero_to == 0) return 0;
  concat_cols_kernel<<<grid_for(rows * zero_to), 256, 0, as_stream(stream)>>>(src, idx, rows, ncols, dst, ld, col0,
                                                                              zero_to);
  PPO_LAUNCH_CHECK("concat_cols_kernel");
  return 0;
}

PPO_API int ppo_rec_indices(const int64_t* envs, int n, int T, int N, int64_t* idx, void* stream) {
  PPO_REQUIRE(n >= 0 && T > 0 && N > 0, "ppo_rec_indices: bad shape");
  if (n == 0) return 0;
  rec_indices_kernel<<<grid_for((long long)T * n), 256, 0, as_stream(stream)>>>(envs, n, T, N, idx);
  PPO_LAUNCH_CHECK("rec_indices_kernel");
  return 0;
}
