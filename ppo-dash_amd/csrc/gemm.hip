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
#include "igemm.h"
#include "igemm_x9.h"
#include "small.h"

namespace {
// ---------------------------------------------------------------------------
// Forward problems
// ---------------------------------------------------------------------------
constexpr int IMG = 84, IMG2 = 84 * 84;
// conv1 forward's LDS image stage: channel stride 7,104 bf16 = 3,552 dwords, which is
// 32 mod 64 (a ds_read_b64 lane's bank is its dword address mod 64), so that the two
// 16-lane halves of a 32-lane group, reading the same rows of channels c and c + 1,
// use complementary banks (see conv1_fwd_bf16x3_body)
constexpr int C1S = 7104;
static_assert(C1S >= IMG2 && (C1S / 2) % 64 == 32, "conv1 stage channel stride");

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
  using Raw = std::conditional_t<sizeof(InT) == 1, uint32_t, f32x4>;
  __device__ Raw a_load(const ACtx& c, int k) const {
    if (!c.ok) return Raw{};
    const int ch = k >> 6, ky = (k >> 3) & 7, kx = k & 7;
    return *reinterpret_cast<const Raw*>(c.base + ch * IMG2 + ky * IMG + kx);
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

// conv1 forward on the bf16 matrix cores, exact (u8 observations, C = 4).
// A pixel u in 0..255 is exact in bf16 and W = W_hi + W_mid + W_lo exactly
// (split_bf16x3), so conv1 = Σ u·W_hi + Σ u·W_mid + Σ u·W_lo where every
// product is exact in fp32 and v_mfma_f32_16x16x32_bf16 accumulates in fp32:
// fp32 arithmetic (as exact per product as v_mfma_f32_*_f32), at 3 bf16 MFMAs
// per 16x16x32 block instead of 8 f32 16x16x4 MFMAs of twice the cycles.
// One persistent block (8 waves) per CU walks images: the image being computed
// sits in LDS as bf16 (4 channels at stride C1S: 56,832 B; two stages), the next
// image is in flight into registers and converted/stored behind the compute.  Wave w:
// output channels 16 * (w & 1) + [0, 16), row tiles {w >> 1, (w >> 1) + 4, ...}
// of 16 output pixels.  k-step s covers channels 2 (s >> 2) + {0, 1} and kernel
// rows 2 (s & 3) + {0, 1}; lane group g = lane >> 4 supplies channel
// 2 (s >> 2) + (g & 1), row 2 (s & 3) + (g >> 1), kx = j = 0..7 — 8 adjacent
// pixels, 16 bytes at an 8-byte-aligned address, read as two ds_read_b64.  Lanes
// 0-31 (g = 0, 1) then read the same rows of two channels C1S apart: each 16-lane
// half covers 32 consecutive dwords mod 64 (16 consecutive output pixels, also
// across an output-row wrap: 4 input rows = 168 dwords = 40 mod 64), the other
// half the complementary 32, so both reads are conflict-free at 2 LDS cycles.
// (Left to itself the compiler merges two 8-byte reads into one ds_read2_b64, 8 LDS
// cycles, MI355X_MICROARCH §LDS; the reads are volatile so that it does not.)
// NPW: weight parts summed (3: exact fp32 weights; 1: half-precision mode, bf16 weights)
// The body takes its LDS (img: two image stages) so that the fused rollout trunk
// (trunk_fwd_kernel) can run it as its first phase in a shared buffer.
template <int C, bool MASK, int NPW = 3>   // MASK: also write the ReLU mask bits (training forward)
__device__ __forceinline__ void conv1_fwd_bf16x3_body(const uint8_t* __restrict__ obs,
                                                      const int64_t* __restrict__ idx, long long row0, int B,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      float* __restrict__ out, uint16_t* __restrict__ mbits,
                                                      uint16_t (*__restrict__ img)[C * C1S]) {
  constexpr int NPX = C * IMG2, CH = NPX / 16, K = C * 64, KS = K / 32, PER = (CH + 511) / 512;
  constexpr int CCH = IMG2 / 16;   // 16-pixel chunks per channel (441)
  static_assert(IMG2 % 16 == 0 && C % 2 == 0, "16-pixel chunks, channel pairs");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ct = wave & 1, rq = wave >> 1;
  const int i16 = lane & 15, g = lane >> 4;
  const int col = ct * 16 + i16;
  const float bv = bias[col];
  // this wave's weight fragments, split once per block: B[k][n] = W[n][k]
  bf16x8 wf[3][KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int c = 2 * (s >> 2) + (g & 1), ky = 2 * (s & 3) + (g >> 1);
    const float* wp = w + (size_t)col * K + c * 64 + ky * 8;
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
  uint4 stage[PER];
  auto fetch = [&](int b) {   // 16 u8 pixels per chunk -> registers
    const uint4* src = reinterpret_cast<const uint4*>(obs + obs_row(idx, row0, b) * (long long)NPX);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = tid + 512 * j;
      if (c < CH) stage[j] = src[c];
    }
  };
  auto put = [&](int buf) {   // u8 -> bf16 (exact: the high half of the fp32 integer), 2 x 16 B stores
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
        const int ch = c / CCH;
        uint4* d = reinterpret_cast<uint4*>(img[buf] + ch * C1S + 16 * (c - ch * CCH));
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
    if (b + G < B) put(cur ^ 1);          // read two iterations ago; the last barrier retired it
    if (b + 2 * G < B) fetch(b + 2 * G);
    // the wave's row tiles rq + 4t: 7 for rq 0, 6 otherwise (25 per image), as a
    // compile-time count, so no MFMA is issued for a tile the wave does not own
    // (with a run-time bound the compiler issued them all and selected: 1,344
    // instead of 1,200 MFMAs per image)
    auto tiles = [&](auto ntc) __attribute__((always_inline)) {
      constexpr int NTL = decltype(ntc)::value;
      const uint16_t* I = img[cur];
      f32x4 acc[NTL];
#pragma unroll
      for (int t = 0; t < NTL; ++t) acc[t] = zero4();
      // this lane's patch origin per row tile (channel g & 1, row g >> 1)
      int pix[NTL];
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int row = (rq + 4 * t) * 16 + i16, oy = row / 20, ox = row - oy * 20;
        pix[t] = (g & 1) * C1S + (g >> 1) * IMG + oy * (4 * IMG) + ox * 4;
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const uint16_t* Is = I + 2 * (s >> 2) * C1S + 2 * (s & 3) * IMG;
        bf16x8 a[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) {   // 8-B aligned: 4ox bf16; volatile: not merged into ds_read2_b64
          typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
          const volatile __attribute__((address_space(3))) u32x2* p2 =
              (const volatile __attribute__((address_space(3))) u32x2*)(Is + pix[t]);
          const u32x2 lo = p2[0], hi = p2[1];
          a[t] = __builtin_bit_cast(bf16x8, uint4{lo.x, lo.y, hi.x, hi.y});
        }
#pragma unroll
        for (int part = 0; part < NPW; ++part)
#pragma unroll
          for (int t = 0; t < NTL; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t], wf[part][s], acc[t], 0, 0, 0);
      }
      float* o = out + (size_t)b * (400 * 32) + col;
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
          const int rt = rq + 4 * t;
          uint64_t bal[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = fmaxf(acc[t][r] * (1.0f / 255.0f) + bv, 0.f);
            o[(rt * 16 + 4 * g + r) * 32] = v;
            if constexpr (MASK) bal[r] = __builtin_amdgcn_ballot_w64(v > 0.f);
          }
          if constexpr (MASK) {   // ReLU mask bits: lane (g, i16) of ballot r -> pixel 16 rt + 4g + r,
            // channel 16 ct + i16; lane j < 16 stores pixel 16 rt + j's 16 bits (one store per tile)
            if (lane < 16) {
              const int r = lane & 3, gg = lane >> 2;
              const uint64_t bsel = r == 0 ? bal[0] : r == 1 ? bal[1] : r == 2 ? bal[2] : bal[3];
              mbits[((size_t)b * 400 + rt * 16 + lane) * 2 + ct] = (uint16_t)(bsel >> (16 * gg));
            }
          }
        }
    };
    if (rq == 0) tiles(std::integral_constant<int, 7>{});
    else tiles(std::integral_constant<int, 6>{});
    __syncthreads();   // every wave is done with img[cur]; img[cur ^ 1] is complete
    cur ^= 1;
  }
}

template <int C, bool MASK, int NPW = 3>
__global__ __launch_bounds__(512) void conv1_fwd_bf16x3_kernel(const uint8_t* __restrict__ obs,
                                                               const int64_t* __restrict__ idx, long long row0,
                                                               int B, const float* __restrict__ w,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ out,
                                                               uint16_t* __restrict__ mbits) {
  __shared__ __attribute__((aligned(16))) uint16_t img[2][C * C1S];
  conv1_fwd_bf16x3_body<C, MASK, NPW>(obs, idx, row0, B, w, bias, out, mbits, img);
}

// conv1 weight gradient on the bf16 matrix cores, exact, part-pipelined
// (ppo_tune_set("conv1_wgrad", 3), default): dW[co][(c,ky,kx)] = Σ_px dz1[px][co] ·
// u[c][4oy+ky][4ox+kx]; the u8 pixels are exact in bf16 and dz = hi + mid + lo
// exactly, so three v_mfma_f32_32x32x16_bf16 per block pair give exact products
// with fp32 accumulation.  Staged so that the staging overlaps
// the MFMAs (a whole-image-stage kernel that filled the LDS measured 2.03-2.10
// ms per minibatch against 1.92-2.01 for this one and was removed):
//   * an image is processed in 5 parts of 4 output rows (80 pixels = 5 k-steps);
//     a part's operands are 42,496 B of LDS — two stages (85 KB) instead of one
//     whole-image stage that fills the LDS;
//       E   [c][20 rows][40 quad slots][4 px] bf16: row yr = input row 16p + yr,
//           slot Q*8 + kx holds u[c][y][16Q + 4j + kx], j = 0..3 (the 4 pixels of
//           an output-row quad for one kx); slot kx bits XOR ((item >> 1) & 7),
//           item = row * 5 + Q, so the staging ds_write_b64 of 16 consecutive
//           items and the B-fragment ds_read_b64 of 32 lanes (4 ky x 8 kx) are
//           both conflict-free
//       dzP [3 planes][32 co][88] bf16: dz of the part split once (no per-wave
//           re-split), 176-B rows: conflict-free ds_read_b128 A fragments
//   * wave w owns one 32-column tile (c = w >> 1, ky = 4 (w & 1) + .., all kx)
//     for every k-step: no k-group partials to combine;
//   * staggered: waves 0-3 stage part i+1 then compute part i, waves 4-7 the
//     other way round, so each SIMD pairs one staging (VALU) wave with one
//     computing (MFMA) wave; the loads of part i+2 are in flight meanwhile.
// One barrier per part.  Output: the split-K slab [Z][32][256] (u8 integers: the
// reduce applies 1/255) and bias partials [Z][32], as the other variants.
// NW = 16 (ppo_tune_set("conv1_wgrad", 4)): four waves per SIMD.  Waves w and
// w + 8 share column tile w & 7 and split the k-steps by parity (wave w + 8 the
// odd global k-steps), their accumulators summed in a fixed order at the end;
// every wave stages at most one item (E items on waves 0-6, dz items on waves
// 8-12), so per SIMD two waves stage while two compute (waves 4-7 and 12-15
// compute first).
// TPW = 2 (NW = 16, ppo_tune_set("conv1_wgrad", 5)): each wave computes two
// column tiles (2 (w & 3), +1) per A fragment read, k-steps split four ways
// (k-group w >> 2 takes global k-steps ≡ w >> 2 mod 4): the dz fragments, the
// same for every tile, are read from LDS half as often (the kernel is LDS-bound:
// the staging writes and the fragment reads share the LDS with each other).
template <int NPD = 3, int NW = 8, int TPW = 1>   // NPD: dz parts summed (3 exact; 1 half-precision mode)
__global__ __launch_bounds__(NW * 64) void conv1_wgrad_parts_kernel(const float* __restrict__ dz1,
                                                                const uint8_t* __restrict__ obs,
                                                                const int64_t* __restrict__ idx, long long row0,
                                                                int B, float* __restrict__ slab,
                                                                float* __restrict__ slab_bias, int dbg) {
  // timing anatomy only (kbench --tune stagger=16*dbg; wrong results): 1 skips the
  // MFMAs, 2 the staging (put), 4 the DMAs, 8 the stagger
  const bool no_mma = dbg & 1, no_put = dbg & 2, no_dma = dbg & 4;
  constexpr int C = 4, NPART = 5, ER = 20, SLOTS = 40, DZS = 88, MAXIMG = 512;
  constexpr int E_BF = C * ER * SLOTS * 4, DZ_BF = 32 * DZS, STG = E_BF + 3 * DZ_BF;   // bf16 elements
  // raw part, as 16-B LDS-DMA pieces: the 4 channels' 20 input rows (4 x 1,680 B =
  // 420 pieces, 16-B aligned in the u8 storage row; 7 wave-instructions, padded to
  // 448) then dz of the part's 80 pixels (10,240 B contiguous = 640 pieces)
  constexpr int EPC = 105, EPIECE = 448, DPIECE = 640, RAWP = EPIECE + DPIECE;
  __shared__ __attribute__((aligned(16))) uint16_t L[2 * STG];           // 84,992 B: two part stages
  __shared__ __attribute__((aligned(16))) uint4 RAW[3][RAWP];            // 52,224 B: raw parts, 3-slot ring
  __shared__ long long rowtab[MAXIMG];                                    // storage row of the block's images
  __shared__ float bred[320];
  static_assert(NW == 8 || NW == 16, "8 or 16 waves");
  static_assert(TPW == 1 || (TPW == 2 && NW == 16), "two tiles per wave with 16 waves");
  constexpr int NT = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  // column tile(s) tile + t (t < TPW); TPW 1: k-step parity kh (NW = 16); TPW 2: k-group kh (0-3)
  const int tile = TPW == 2 ? 2 * (wave & 3) : wave & 7, kh = TPW == 2 ? wave >> 2 : wave >> 3;
  const int G = gridDim.x;
  const int nimg = blockIdx.x < B ? (B - 1 - (int)blockIdx.x) / G + 1 : 0, nit = NPART * nimg;
  for (int k = tid; k < nimg; k += NT) rowtab[k] = obs_row(idx, row0, (int)blockIdx.x + k * G);
  // B column of this lane: n = 32 (tile + t) + l32 -> (c, ky, kx)
  int qoff[TPW][5][2];   // E element offset of the lane's quads for local k-step ls
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tt = tile + t, bc = tt >> 1, bky = 4 * (tt & 1) + (l32 >> 3), bkx = l32 & 7;
#pragma unroll
    for (int ls = 0; ls < 5; ++ls)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ql = 4 * ls + 2 * h + j, oyl = ql / 5, Q = ql - 5 * oyl;
        const int r = bc * ER + 4 * oyl + bky, item = r * 5 + Q;
        qoff[t][ls][j] = (r * SLOTS + Q * 8 + (bkx ^ ((item >> 1) & 7))) * 4;
      }
  }
  const int aoff = E_BF + l32 * DZS + 8 * h;   // + plane * DZ_BF + 16 ls
  // staging items: E item tid < 400 (row r = tid / 5 = c * 20 + yr, quad Q = tid % 5);
  // dz item tid < 320 (co = tid & 31, pixel octet oc = tid >> 5).  Threads without
  // an item DMA item 0's addresses (harmless duplicates) so every wave issues the
  // same DMA count.
  const bool e_on = tid < 400, d_on = NW == 8 ? tid < 320 : tid >= 512 && tid < 832;
  const int eit = e_on ? tid : 0, dit = d_on ? tid - (NW == 8 ? 0 : 512) : 0;
  const int er = eit / 5, eQ = eit - 5 * er, ec = er / ER, eyr = er - ER * ec, ef = (eit >> 1) & 7;
  const int dco = dit & 31, doc = dit >> 5;
  float bacc = 0.f;
  // DMA of item j's raw part into RAW[j & 1]: wave w moves pieces 64 w + lane of
  // the image rows (waves 0-6) and of dz (pieces 64 (w + 8 i) + lane, i = 0, 1)
  auto dma = [&](int j) {
    if (no_dma) return;
    const int jj = j < nit ? j : nit - 1, k = jj / NPART, p = jj - NPART * k, b = (int)blockIdx.x + k * G;
    uint4* dst = RAW[jj % 3];
    if (wave < 7) {
      const int piece = min(64 * wave + lane, C * EPC - 1), c = piece / EPC, r = piece - EPC * c;
      const uint8_t* src = obs + rowtab[k] * (long long)(C * IMG2) + c * IMG2 + p * (16 * IMG) + 16 * r;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                       reinterpret_cast<__attribute__((address_space(3))) void*>(
                                           reinterpret_cast<uintptr_t>(dst + 64 * wave)), 16, 0, 0);
    }
    const char* dsrc = reinterpret_cast<const char*>(dz1 + (size_t)b * 12800 + p * 80 * 32);
#pragma unroll
    for (int i = 0; i < (NW == 8 ? 2 : 1); ++i) {
      const int blk = NW == 8 ? wave + 8 * i : wave - 6;   // wave-uniform; NW = 16: waves 6-15
      if (blk >= 0 && blk < DPIECE / 64)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(dsrc + 16 * (64 * blk + lane)),
                                         reinterpret_cast<__attribute__((address_space(3))) void*>(
                                             reinterpret_cast<uintptr_t>(dst + EPIECE + 64 * blk)), 16, 0, 0);
    }
  };
  auto put = [&](int j, int st) {   // item j: RAW[j % 3] -> stage st
    if (no_put) return;
    const uint32_t* R = reinterpret_cast<const uint32_t*>(RAW[j % 3]);
    uint32_t ew[5];
    float dv[8];
    if (NW == 8 || e_on) {   // NW = 8: every thread reads both (all loads issued first)
#pragma unroll
      for (int q = 0; q < 5; ++q) ew[q] = R[(ec * 1680 + eyr * IMG + 16 * eQ) / 4 + q];
    }
    if (NW == 8 || d_on) {
#pragma unroll
      for (int q = 0; q < 8; ++q) dv[q] = __uint_as_float(R[4 * EPIECE + (8 * doc + q) * 32 + dco]);
    }
    uint16_t* S = L + st * STG;
    if (e_on) {
#pragma unroll
      for (int kx = 0; kx < 8; ++kx) {   // u[16Q + 4i + kx] = byte (kx & 3) of dword i + (kx >> 2)
        const int o = kx >> 2, sh = 8 * (kx & 3);
        float f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = (float)((ew[i + o] >> sh) & 255u);
        const uint2 q = {__builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u),
                         __builtin_amdgcn_perm(__float_as_uint(f[3]), __float_as_uint(f[2]), 0x07060302u)};
        *reinterpret_cast<uint2*>(S + (er * SLOTS + eQ * 8 + (kx ^ ef)) * 4) = q;
      }
    }
    if (d_on) {
      Frag3 fr;
      split8(f32x4{dv[0], dv[1], dv[2], dv[3]}, f32x4{dv[4], dv[5], dv[6], dv[7]}, fr, NPD == 1);
      uint16_t* d = S + E_BF + dco * DZS + 8 * doc;
      *reinterpret_cast<bf16x8*>(d) = fr.h;
      if constexpr (NPD == 3) {
        *reinterpret_cast<bf16x8*>(d + DZ_BF) = fr.m;
        *reinterpret_cast<bf16x8*>(d + 2 * DZ_BF) = fr.l;
      }
      bacc += ((dv[0] + dv[1]) + (dv[2] + dv[3])) + ((dv[4] + dv[5]) + (dv[6] + dv[7]));
    }
  };
  f32x16 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  auto compute = [&](int st, int i) {
    if (no_mma) return;
    const uint16_t* S = L + st * STG;
#pragma unroll
    for (int ls = 0; ls < 5; ++ls) {   // global k-step 5 i + ls; the skips are wave-uniform
      if (TPW == 2 && ((i + ls) & 3) != kh) continue;
      if (TPW == 1 && NW == 16 && ((i + ls) & 1) != kh) continue;
      bf16x8 bq[TPW];
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const uint2 q1 = *reinterpret_cast<const uint2*>(S + qoff[t][ls][0]);
        const uint2 q2 = *reinterpret_cast<const uint2*>(S + qoff[t][ls][1]);
        bq[t] = __builtin_bit_cast(bf16x8, uint4{q1.x, q1.y, q2.x, q2.y});
      }
      const uint16_t* A = S + aoff + 16 * ls;
      if constexpr (NPD == 3) {
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(A + 2 * DZ_BF), am = *reinterpret_cast<const bf16x8*>(A + DZ_BF);
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bq[t], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bq[t], acc[t], 0, 0, 0);
        }
      }
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(A);
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bq[t], acc[t], 0, 0, 0);
    }
  };
  // pipeline: item j's pieces are DMA'd into RAW[j % 3] at item j - 3 (by every
  // wave, a share each); at the end of item j - 2 every wave waits for its own
  // share (vmcnt = one item's DMA count: item j + 1's may stay in flight) and the
  // barrier publishes the slot; item j - 1 stages it (put) into LDS stage j & 1.
  const int nops = NW == 8 ? (wave < 7 ? 1 : 0) + 1 + (wave + 8 < DPIECE / 64 ? 1 : 0)
                            : (wave < 7 ? 1 : 0) + (wave >= 6 ? 1 : 0);
  auto wait_raw = [&]() {   // all but the youngest item's DMAs retired
    if (nops == 3) __builtin_amdgcn_s_waitcnt(0x0F73);        // vmcnt(3)
    else if (nops == 2) __builtin_amdgcn_s_waitcnt(0x0F72);   // vmcnt(2)
    else __builtin_amdgcn_s_waitcnt(0x0F71);                  // vmcnt(1)
  };
  // block barrier that does not drain the in-flight DMAs (__syncthreads' release
  // fence would wait for them: vmcnt(0)); LDS stores are retired by lgkmcnt(0),
  // and the memory clobber keeps the compiler from moving LDS accesses across it
  auto part_barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  __syncthreads();   // rowtab
  if (nit > 0) {
    dma(0);
    dma(1);
    dma(2);
    if (nops == 3) __builtin_amdgcn_s_waitcnt(0x0F76);        // vmcnt(6): item 0 retired
    else if (nops == 2) __builtin_amdgcn_s_waitcnt(0x0F74);   // vmcnt(4)
    else __builtin_amdgcn_s_waitcnt(0x0F72);                  // vmcnt(2)
    part_barrier();
    put(0, 0);
    wait_raw();   // item 1 retired (item 2 may be in flight)
  }
  part_barrier();
  const bool late = (NW == 8 ? wave >= 4 : ((wave >> 2) & 1) != 0) && !(dbg & 8);
  for (int i = 0; i < nit; ++i) {
    const int st = i & 1;
    const bool more = i + 1 < nit;
    if (!late && more) put(i + 1, st ^ 1);
    if (more) dma(i + 3);   // into RAW[i % 3]: item i was staged before the last barrier
    compute(st, i);
    if (late && more) put(i + 1, st ^ 1);
    wait_raw();   // item i + 2 retired (item i + 3 may be in flight)
    part_barrier();
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // drain the clamped tail DMAs before the block exits
  float* X = reinterpret_cast<float*>(L);   // stage space, free now: k-group partials
  if constexpr (NW == 16 && TPW == 1) {   // odd-k-step partials added to the even ones
    if (kh) {
#pragma unroll
      for (int r = 0; r < 16; ++r) X[(r * 8 + tile) * 64 + lane] = acc[0][r];
    }
    __syncthreads();
    if (!kh) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][r] += X[(r * 8 + tile) * 64 + lane];
    }
  }
  if constexpr (TPW == 2) {   // fixed order: (k0 + k2) + (k1 + k3); slot = tile pair (+ 4)
    auto xo = [&](int slot, int t, int r) { return ((slot * 2 + t) * 16 + r) * 64 + lane; };
    const int tp = wave & 3;
    if (kh >= 2) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[xo((kh - 2) * 4 + tp, t, r)] = acc[t][r];
    }
    __syncthreads();
    if (kh < 2) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += X[xo(kh * 4 + tp, t, r)];
    }
    __syncthreads();
    if (kh == 1) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[xo(tp, t, r)] = acc[t][r];
    }
    __syncthreads();
    if (kh == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += X[xo(tp, t, r)];
    }
  }
  float* out = slab + (size_t)blockIdx.x * 32 * 256;
  if (kh == 0) {
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = (r & 3) + 8 * (r >> 2) + 4 * h, n = 32 * (tile + t) + l32;
        out[co * 256 + n] = acc[t][r];
      }
  }
  if (d_on) bred[dit] = bacc;
  __syncthreads();
  if (tid < 32) {   // channel tid: its 10 pixel octets, fixed order
    float t = 0.f;
#pragma unroll
    for (int o = 0; o < 10; ++o) t += bred[32 * o + tid];
    slab_bias[(size_t)blockIdx.x * 32 + tid] = t;
  }
}

// ReLU mask bits of a conv1 output [B][400][32]: bit c of word p = (a1[p][c] > 0),
// for the conv1 paths without the fused epilogue (one thread per half pixel).
__global__ __launch_bounds__(256) void relu_bits_kernel(const float* __restrict__ a1, long long halves,
                                                        uint16_t* __restrict__ mbits) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < halves; i += (long long)gridDim.x * 256) {
    const f32x4* p = reinterpret_cast<const f32x4*>(a1 + 16 * i);
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = p[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) m |= (v[e] > 0.f ? 1u : 0u) << (4 * q + e);
    }
    mbits[i] = (uint16_t)m;
  }
}

// ---------------------------------------------------------------------------
// Image-resident conv2 / conv3 kernels on the bf16 matrix cores (exact split,
// DESIGN.md §3): forward, input gradient (the epilogue applies the ReLU mask of
// the layer below, threshold_backward: pass where the saved output is > 0) and
// weight gradient.
// ---------------------------------------------------------------------------
// conv2 forward, image-resident on the bf16 matrix cores (exact split, DESIGN.md
// §3), two LDS stages: a2[b][m][co] =
// relu(b2[co] + Σ_k im2col(a1)[m][k] W2p[co][k]), m = (oy, ox), k = (ky, kx, ci).
// One persistent block (8 waves) per CU walks images.  Wave w: n tile w & 3 (16
// co), taps 8 (w >> 2) .. +7 (ky rows 0-1 / 2-3), its weight fragments
// (pre-split planes) in registers; the two K halves are summed through LDS.  The
// next image's split is staged into the second stage *during* the current
// image's k-steps instead of in a phase of its own (the single-stage kernel this
// replaced, 1.98 ms per minibatch, and an LDS-DMA staged variant, 2.00 ms, were
// removed; this one is bit-identical to both).
//   * Compact parity layout, 400 16-B units per 8-channel chunk: pixel (y, x) at
//     P = 100 (2 (y & 1) + (x & 1)) + 10 (y >> 1) + (x >> 1), so tap (ky, kx) of
//     output pixel (oy, ox) reads v + toff(ky, kx), v = 10 oy + ox.  Row i of row
//     tile t is the t-th pixel (by v) with v ≡ i (mod 16) (≤ 6 per residue: 6
//     tiles; a missing one is a dummy row reading pixel v = i): the 16 lanes of
//     a ds_read_b128 group read 16 distinct residues, conflict-free.  That leaves
//     five real rows in the sixth tile (v = 80 .. 88: the sixth pixels of residues
//     0, 2, 4, 6, 8).  MT = 5 (the standalone launches): residues 9, 11, 13, 15 have
//     four pixels, so tile 4's rows 9, 11, 13, 15 take v = 82, 84, 86, 88 (a 2-way
//     bank conflict in that tile's reads), and v = 80 (output (8, 0)) is left to
//     conv2_fwd_lone_kernel, 16 images per tile; the fused trunk keeps MT = 6.  Two stages
//     x 3 planes x 4 chunks x 400 x 16 B = 153,600 B.
//   * The K-half partials (24,576 B) are handed over in the lo plane of the stage
//     the image has just left: kh 1 writes them after barrier A, kh 0 reads them
//     after barrier B; the next image's hi / mid parts are staged into that
//     stage's planes 0-1 during k-steps 0-3, its lo parts held in registers
//     until a mid-image barrier (after k-step 5) has retired the partial reads,
//     then written during k-steps 6-7.  The image after next is fetched into
//     registers one unit per k-step (1-4), each once its register has been staged.
//   * Epilogue in the swapped MFMA orientation (weights as A): one 16-B store of
//     four consecutive channels per tile, dummy rows dropped by buffer range.
// DBG (timing anatomy of a diagnostic build only — the library instantiates DBG = 0;
// wrong results): 1 skips the MFMAs, 2 the staging (split + ds_write), 4 the global
// loads, 8 the epilogue stores (profiles/r04_c2f_anatomy_kbench.log)
constexpr int C2F_STG = 3 * 4 * 400, C2F_MT = 6;   // conv2 forward: bf16x8 units per stage, row tiles
constexpr int C2F_LDS = 2 * C2F_STG * 16 + 2 * C2F_MT * 16 * 4;   // stages + vtab + otab (154,368 B)
template <int NP, bool MASK>
__device__ __forceinline__ void conv2_lone_tiles(const float* __restrict__ a1, const bf16x8 (&bw)[8][3],
                                                 const float* __restrict__ bias, float* __restrict__ out,
                                                 uint16_t* __restrict__ mbits, uint8_t* __restrict__ lds,
                                                 long long base, long long stride, int nimg, int t0, int tstep);
template <int NP, bool MASK = false, int DBG = 0, int MT = C2F_MT, bool LONE = false>
__device__ __forceinline__ void conv2_fwd_x9c_body(const float* __restrict__ a1, int B,
                                                   const uint16_t* __restrict__ wpl, const float* __restrict__ bias,
                                                   float* __restrict__ out, uint16_t* __restrict__ mbits,
                                                   uint8_t* __restrict__ lds) {
  constexpr int U = 400, PLN = 4 * U, STG = 3 * PLN, KS = 8, WN = 64 * 512;
  static_assert(MT == 5 || MT == 6, "row tiles: 6, or 5 with the lone pixel elsewhere");
  constexpr int UNITS = 4 * U, UPER = (UNITS + 511) / 512;   // 4 units per thread (the 4th: wave 0)
  static_assert(STG == C2F_STG, "stage size");
  bf16x8* const S = reinterpret_cast<bf16x8*>(lds);
  int (*const vtab)[16] = reinterpret_cast<int (*)[16]>(lds + 2 * STG * 16);
  int (*const otab)[16] = reinterpret_cast<int (*)[16]>(lds + 2 * STG * 16 + MT * 16 * 4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int nt = wave & 3, kh = wave >> 2, co = 16 * nt + i16;
  if (tid < 16) {
    int t = 0;
    for (int v = tid; v <= 88; v += 16)
      if (v % 10 != 9 && t < MT) {
        vtab[t][tid] = v;
        otab[t][tid] = 9 * (v / 10) + v % 10;
        ++t;
      }
    if (MT == 5 && t == 4) {   // residues 9, 11, 13, 15 (4 pixels each) take the sixth pixels
      // of residues 2, 4, 6, 8 (v = 82 .. 88; a 2-way bank conflict in tile 4's reads);
      // residue 0's (v = 80) is the lone pixel
      const int v = 82 + (tid - 9);
      vtab[4][tid] = v;
      otab[4][tid] = 9 * (v / 10) + v % 10;
      t = 5;
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
  // staging unit u = tid + 512 j: chunk c = (u >> 3) & 3 of the pixel at compact
  // position rho = 8 (u >> 5) + (u & 7): 8 consecutive lanes write 8 consecutive
  // units (conflict-free ds_write_b128) and 4 lanes read one pixel's 128-B line
  int usrc[UPER], udst[UPER];
#pragma unroll
  for (int j = 0; j < UPER; ++j) {
    const int u = min(tid + 512 * j, UNITS - 1), rho = 8 * (u >> 5) + (u & 7), c = (u >> 3) & 3;
    const int par = rho / 100, rem = rho - 100 * par, yh = rem / 10, xh = rem - 10 * yh;
    const int y = 2 * yh + (par >> 1), x = 2 * xh + (par & 1);
    usrc[j] = (y * 20 + x) * 8 + 2 * c;
    udst[j] = c * U + rho;
  }
  const bool has_last = tid + 512 * (UPER - 1) < UNITS;
  f32x4 stg[UPER][2];
  bf16x8 lo[UPER];
  auto fetch_unit = [&](int b, int j) {   // unconditional (the 4th unit of waves 1-7 reloads unit 1599)
    if constexpr ((DBG & 4) != 0) {   // no load; the registers stay opaque to the compiler
      asm volatile("" : "+v"(stg[j][0]), "+v"(stg[j][1]));
      return;
    }
    const f32x4* src = reinterpret_cast<const f32x4*>(a1 + (size_t)b * 12800);
    stg[j][0] = src[usrc[j]];
    stg[j][1] = src[usrc[j] + 1];
  };
  auto fetch = [&](int b) {
#pragma unroll
    for (int j = 0; j < UPER; ++j) fetch_unit(b, j);
  };
  auto put_hm = [&](int j, int st) {   // hi / mid parts now, lo part held
    if constexpr ((DBG & 2) != 0) {   // no staging; the loaded registers stay live
      asm volatile("" ::"v"(stg[j][0]), "v"(stg[j][1]));
      return;
    }
    Frag3 f;
    split8(stg[j][0], stg[j][1], f, NP == 1);
    lo[j] = f.l;
    if (j < UPER - 1 || has_last) {
      bf16x8* d = S + st * STG + udst[j];
      d[0] = f.h;
      if constexpr (NP > 1) d[PLN] = f.m;
    }
  };
  auto put_l = [&](int j, int st) {
    if constexpr ((DBG & 2) != 0) return;
    if constexpr (NP > 1)
      if (j < UPER - 1 || has_last) S[st * STG + 2 * PLN + udst[j]] = lo[j];
  };
  // block barrier that leaves the image prefetch in flight (__syncthreads' fence
  // would drain every outstanding load): LDS ops retired, compiler fence
  auto lds_barrier = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  __syncthreads();   // vtab / otab
  int vrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) vrow[t] = vtab[t][i16] + g * U;
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
#pragma unroll
    for (int j = 0; j < UPER; ++j) {
      put_hm(j, 0);
      put_l(j, 0);
    }
    fetch(b + G < B ? b + G : b);
  }
  __syncthreads();
  for (; b < B; b += G) {
    // no branches in the k loop (a conditional load or stage write made the wait
    // counts unknown at the merge: vmcnt(0) at every staging step): past the
    // block's last image the staging re-reads / re-stages an image nothing uses
    const int bnn = b + 2 * G < B ? b + 2 * G : b;
    const bf16x8* Sc = S + cur * STG;
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = zero4();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int tap = 8 * kh + s, ky = tap >> 2, kx = tap & 3;
      const int toff = 100 * (2 * (ky & 1) + (kx & 1)) + 10 * (ky >> 1) + (kx >> 1);
      const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
#pragma unroll
      for (int t0 = 0; t0 < MT; t0 += 3) {
        Frag3 a[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          if (t0 + u >= MT) continue;
          const bf16x8* q = Sc + vrow[t0 + u] + toff;
          a[u].h = q[0];
          if constexpr (NP > 1) {
            a[u].m = q[PLN];
            a[u].l = q[2 * PLN];
          }
        }
#define PPO_PART(X, Y) \
  _Pragma("unroll") for (int u = 0; u < 3; ++u) if (t0 + u < MT) acc[t0 + u] = mma(w.Y, a[u].X, acc[t0 + u]);
        if constexpr ((DBG & 1) == 0) {
          PPO_PRODUCTS(NP, PPO_PART)
        } else {   // keep the fragment reads live
#pragma unroll
          for (int u = 0; u < 3; ++u)
            if (t0 + u < MT) asm volatile("" ::"v"(a[u].h), "v"(a[u].m), "v"(a[u].l));
        }
#undef PPO_PART
      }
      if (s < UPER) put_hm(s, cur ^ 1);
      // the image after next, one unit per k-step as its registers free up (all
      // four at one k-step stalled every wave of the chip at the same time)
      if (s >= 1 && s <= UPER) fetch_unit(bnn, s - 1);
      if (s == 5) lds_barrier();   // mid-image: the previous image's partials (lo plane of stage cur ^ 1) are read
      if (s >= 6) {
#pragma unroll
        for (int j = 0; j < UPER; ++j)
          if ((j & 1) == s - 6) put_l(j, cur ^ 1);
      }
    }
    lds_barrier();   // A: stage cur consumed; stage cur ^ 1 complete
    f32x4* R = reinterpret_cast<f32x4*>(S + cur * STG + 2 * PLN);   // partials in the lo plane just left
    if (kh == 1) {
#pragma unroll
      for (int t = 0; t < MT; ++t) R[(nt * MT + t) * 64 + lane] = acc[t];
    }
    lds_barrier();   // B: partials in LDS
    if (kh == 0) {
      const auto rs = make_rsrc(out + (size_t)b * (81 * 64), 81 * 64 * 4);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const f32x4 v = acc[t] + R[(nt * MT + t) * 64 + lane];
        const int m = otab[t][i16];
        f32x4 y;
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + bv4[r], 0.f);
        if constexpr ((DBG & 8) == 0) bstore_f32x4(y, rs, m >= 0 ? 4 * (m * 64 + 16 * nt + 4 * g) : -1);
        if constexpr (MASK && (DBG & 8) == 0) {   // ReLU mask bits of pixel m, channels 16 nt .. +15: 4 lanes' nibbles
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
  if constexpr (MT == 5 && LONE) {
    // the lone pixel (output 72) of this block's own images, 16 per tile, after its
    // image loop (round 6, VERDICT r05 item 7: no separate launch; the weight
    // fragments are the ones the image loop used)
    __syncthreads();   // the last image's K-half partials (in the LDS) are read
    const int blk = blockIdx.x;
    const int nimg = blk < B ? (B - 1 - blk) / G + 1 : 0;
    conv2_lone_tiles<NP, MASK>(a1, bw, bias, out, mbits, lds, blk, G, nimg, 0, 1);
  }
}

#ifndef C2F_LONE
// standalone conv2 forward: 1 five row tiles + conv2_fwd_lone_kernel (default), 2 the
// lone pixel inside the same launch after each block's image loop, 0 six tiles.
// Round 6 measured 2 against 1 on one box, alternating
// (profiles/r06_d_lone_trunk_kbab.log): 1.804-1.817 vs 1.787-1.789 ms (conv2_fwd),
// 1.746-1.754 vs 1.740-1.744 ms (the masked training form) — the separate launch
// runs two 70-KB-LDS blocks per CU (16 waves) where the folded tiles run at the
// tail of one 8-wave block per CU, so it stays.  The fused trunk folds them (one
// tile per block at the rollout's 16 images per block, no extra launch).
#define C2F_LONE 1
#endif
template <int NP, bool MASK = false, int DBG = 0>
__global__ __launch_bounds__(512) void conv2_fwd_x9c_kernel(const float* __restrict__ a1, int B,
                                                           const uint16_t* __restrict__ wpl,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ out,
                                                           uint16_t* __restrict__ mbits) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[C2F_LDS];
  conv2_fwd_x9c_body<NP, MASK, DBG, C2F_LONE ? 5 : 6, C2F_LONE == 2>(a1, B, wpl, bias, out, mbits, lds);
}

// conv2 forward of output pixel 72 = (8, 0) (phase-grid v = 80, the sixth row tile's
// only real row) for 16 images per tile.  The tile's 16 patches (a1 rows 16-19, columns 0-3: 4 x 512 contiguous bytes
// per image, 32 KB per tile) are loaded once per block — each thread four 16-B
// pieces, the next tile's in registers during this tile's MFMAs — and staged in LDS
// (two stages; image rows padded by 16 B so the 16 images of a fragment read hit
// distinct banks): loading them per wave moved each chunk four times through the
// L2, 107 vs 76 µs per 65,536 images (profiles/r05_zr_lone_anatomy.txt; two tiles
// of loads in flight measured no faster).  The same operands as conv2_fwd_x9c_body's
// (the same split8 of the same 8-channel chunks, the same weight planes), the same
// MFMA sequence per wave (k-steps of its K half in order, parts in PPO_PRODUCTS
// order), the K halves summed kh 0 + kh 1, the same epilogue: an MFMA output column
// depends only on its own B column, so the result is bit-identical to a six-tile
// launch whichever images share a tile (test_trunk_fwd_equals_three_launches; the
// six-tile form is C2F_LONE = 0).
// Tiles t0, t0 + tstep, ... of the images base + stride * i (i < nimg, 16 per tile:
// row i16 of the B operand is image base + stride * (16 t + i16)).  The kernel above
// runs it after its image loop over the block's own images (base = blockIdx.x, stride
// = the grid), conv2_fwd_lone_kernel (C2F_LONE = 1) over contiguous images.
// Round 6: the patches are split into their bf16 planes once, while staged (each thread
// one 8-channel chunk of one image), instead of by every wave at fragment read (the 4
// waves of a K half split the same chunks: 7 split VALU per MFMA).
constexpr int C2L_IR = 65;    // 16-B units per staged image row and plane (64 + pad: the 16
                              // images of a fragment read hit distinct 16-B slots)
constexpr int C2L_PL = 16 * C2L_IR;   // units per plane
constexpr int C2L_LDS = 2 * 3 * C2L_PL * 16 + 4 * 64 * 16;   // two 3-plane stages + K-half partials (103,936 B)
static_assert(C2L_LDS <= C2F_LDS, "the lone tiles reuse the image loop's LDS");
template <int NP, bool MASK>
__device__ __forceinline__ void conv2_lone_tiles(const float* __restrict__ a1, const bf16x8 (&bw)[8][3],
                                                 const float* __restrict__ bias, float* __restrict__ out,
                                                 uint16_t* __restrict__ mbits, uint8_t* __restrict__ lds,
                                                 long long base, long long stride, int nimg, int t0, int tstep) {
  constexpr int KS = 8, M = 72, IR = C2L_IR, PL = C2L_PL;
  uint4 (*const P)[3 * PL] = reinterpret_cast<uint4 (*)[3 * PL]>(lds);
  f32x4* const R = reinterpret_cast<f32x4*>(lds + 2 * 3 * PL * 16);
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = wave & 3, kh = wave >> 2;
  const int ntile = (nimg + 15) / 16;
  // chunk c = tid + 512 j (j < 2) of a tile: image c >> 6, 8-channel chunk u = c & 63 of
  // its patch = tap (4 ky + kx) * 4 + channel octet; a1 offset (16 + ky) * 640 + (u & 15) * 8
  f32x4 pc[2][2];
  auto fetch = [&](int T) {   // past the last tile / image: zeros, nothing loaded
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 512 * j, im = c >> 6, u = c & 63, i = 16 * T + im;
      const bool live = T < ntile && i < nimg;
      const float* src = a1 + (size_t)(base + stride * (live ? i : 0)) * 12800 + (16 + (u >> 4)) * 640 + (u & 15) * 8;
      pc[j][0] = live ? *reinterpret_cast<const f32x4*>(src) : zero4();
      pc[j][1] = live ? *reinterpret_cast<const f32x4*>(src + 4) : zero4();
    }
  };
  auto put = [&](int st) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + 512 * j, o = (c >> 6) * IR + (c & 63);
      Frag3 f;
      split8(pc[j][0], pc[j][1], f, NP == 1);
      P[st][o] = __builtin_bit_cast(uint4, f.h);
      if constexpr (NP != 1) {
        P[st][PL + o] = __builtin_bit_cast(uint4, f.m);
        P[st][2 * PL + o] = __builtin_bit_cast(uint4, f.l);
      }
    }
  };
  fetch(t0);
  put(0);
  __syncthreads();
  int cur = 0;
  for (int T = t0; T < ntile; T += tstep) {
    fetch(T + tstep);
    const int i = 16 * T + i16;
    const bool live = i < nimg;
    const long long b = base + stride * (long long)i;
    f32x4 acc = zero4();
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int o = i16 * IR + (8 * kh + s) * 4 + g;
      Frag3 a;
      a.h = __builtin_bit_cast(bf16x8, P[cur][o]);
      if constexpr (NP != 1) {
        a.m = __builtin_bit_cast(bf16x8, P[cur][PL + o]);
        a.l = __builtin_bit_cast(bf16x8, P[cur][2 * PL + o]);
      }
      const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
#define PPO_PART(X, Y) acc = mma(w.Y, a.X, acc);
      PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
    }
    if (kh == 1) R[nt * 64 + lane] = acc;
    put(cur ^ 1);   // the stage read one tile ago (the last barrier retired its reads)
    __syncthreads();   // partials in R; stage cur ^ 1 complete
    if (kh == 0) {
      const f32x4 bv4 = *reinterpret_cast<const f32x4*>(bias + 16 * nt + 4 * g);
      const f32x4 v = acc + R[nt * 64 + lane];
      f32x4 y;
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + bv4[r], 0.f);
      if (live) *reinterpret_cast<f32x4*>(out + (size_t)b * (81 * 64) + M * 64 + 16 * nt + 4 * g) = y;
      if constexpr (MASK) {
        int nib = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) nib |= (y[r] > 0.f ? 1 : 0) << r;
        const int w16 = nib | (__shfl_down(nib, 16, 64) << 4) | (__shfl_down(nib, 32, 64) << 8) |
                        (__shfl_down(nib, 48, 64) << 12);
        if (g == 0 && live) mbits[((size_t)b * 81 + M) * 4 + nt] = (uint16_t)w16;
      }
    }
    __syncthreads();   // R read before the next tile's partials
    cur ^= 1;
  }
}

template <int NP, bool MASK>
__global__ __launch_bounds__(512) void conv2_fwd_lone_kernel(const float* __restrict__ a1, int B,
                                                             const uint16_t* __restrict__ wpl,
                                                             const float* __restrict__ bias,
                                                             float* __restrict__ out,
                                                             uint16_t* __restrict__ mbits) {
  constexpr int KS = 8, WN = 64 * 512;
  __shared__ __attribute__((aligned(16))) uint8_t lds[C2L_LDS];
  const int tid = threadIdx.x, i16 = tid & 15, g = (tid & 63) >> 4, wave = tid >> 6;
  const int co = 16 * (wave & 3) + i16, kh = wave >> 2;
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + co * 512 + (8 * kh + s) * 32 + 8 * g);
  conv2_lone_tiles<NP, MASK>(a1, bw, bias, out, mbits, lds, 0, 1, B, blockIdx.x, gridDim.x);
}

// conv2 weight gradient, image-resident on the bf16 matrix cores (exact split,
// DESIGN.md §3): dW2[co][k] = Σ_pixels dz2[m][co] · a1[2oy+ky][2ox+kx][ci],
// k = (ky, kx, ci); per image a 64 x 512 x 81 product (reduction padded to 96 =
// 3 k-steps of 32), accumulated in registers over the block's images and
// written once as the block's split-K partial (slab [Z][64][512], bias
// partials [Z][64]; ppo_wgrad_reduce sums the Z partials in a fixed order).
// Per image the LDS holds, split into bf16 planes (the next image in flight in
// registers, stored between compute phases):
//   X  [3][400 px][32 ci]  a1, pixels in parity order Q = 20 y + 10 (x & 1) + (x >> 1)
//                          (76,800 B): the B fragment (8 reduction slots x 16 ci of
//                          one tap) comes from two ds_read_b64_tr_b16 per plane —
//                          4 pixel rows each, gathered by per-lane row addresses;
//                          8-B unit u of pixel Q at u ^ 4 ((Q >> 3) & 1)
//   D  [3][64 co][112]     dz2 transposed to [co][reduction slot] (43,008 B; rows of
//                          14 16-B units: conflict-free ds_read_b128 A fragments)
// Reduction slot r -> pixel: the 72 pixels with ox < 8 oy-major, then the ox = 8
// column (no 4-slot tr group straddles an output row; fewer bank conflicts);
// slots 81..95 have dz = 0 and read pixel 80's finite a1.
// Wave w: k columns 64 w .. +63 (taps 2w, 2w+1, both ci halves) x all 64 co:
// 16 accumulator tiles (64 VGPRs).
__device__ __forceinline__ int c2w_pix(int r) {
  r = r < 80 ? r : 80;
  return r < 72 ? (r >> 3) * 9 + (r & 7) : (r - 72) * 9 + 8;
}

// DBG (timing anatomy of a diagnostic build only — the library instantiates DBG = 0;
// wrong results): 1 skips the MFMAs, 2 the LDS staging (split + ds_write), 4 the global loads; schedule
// experiments (right results): 8 spreads the 8 load parts over all 12 slots, 16
// starts every block at once (no s_sleep stagger of the odd blocks)
template <int NP, int DBG = 0>
__global__ __launch_bounds__(512) void conv2_wgrad_x9_kernel(const float* __restrict__ dz2,
                                                            const float* __restrict__ a1, int B,
                                                            float* __restrict__ slab,
                                                            float* __restrict__ slab_bias) {
  constexpr int XPL = 400 * 32, DR = 112, DPL = 64 * DR;
  constexpr int XU = 1600, XPER = (XU + 511) / 512, DU = 64 * 12, DPER = (DU + 511) / 512;
  __shared__ __attribute__((aligned(16))) uint16_t X[3 * XPL];
  __shared__ __attribute__((aligned(16))) uint16_t D[3 * DPL];
  __shared__ float bred[512];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int q = i16 >> 2, p = i16 & 3;
  // tap-(0,0) pixel (parity order) of the row this lane addresses in the tr
  // reads of k-step s, half h: Q = Qb + 20 ky + 10 (kx & 1) + (kx >> 1)
  int Qb[3][2];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = c2w_pix(32 * s + 8 * g + 4 * h + q), oy = m / 9;
      Qb[s][h] = 40 * oy + (m - 9 * oy);
    }
  // staging maps: X unit u -> (pixel Q = u >> 2, 16-B chunk c = u & 3); D unit
  // v -> (co = v & 63, slots 8 (v >> 6) .. +7)
  int xsrc[XPER], xdst[XPER];
#pragma unroll
  for (int j = 0; j < XPER; ++j) {
    const int u = tid + 512 * j, Q = u >> 2, c = u & 3, y = Q / 20, rem = Q - 20 * y;
    const int x = rem < 10 ? 2 * rem : 2 * (rem - 10) + 1;
    xsrc[j] = (y * 20 + x) * 32 + 8 * c;
    xdst[j] = Q * 32 + 8 * (c ^ (((Q >> 3) & 1) * 2));
  }
  f32x4 xs[XPER][2];
  float ds[DPER][8];
  float bsum = 0.f;   // bias partial of co = tid & 63 (fixed for this thread's D units)
  // the next image's loads in 8 parts (a1 units j = 0..3, then dz2 units j = 0, 1
  // in halves), issued one per (k-step, n tile) slot of the first two k-steps of
  // the current image's MFMAs: issued between the barriers, with every CU at the
  // same point, the 72 KB per image stalled the waves at issue for the whole
  // chip's transfer time (tools/kbench.py conv2_wgrad_anat*: 0.66 of 1.78 ms)
  auto fetch_part = [&](int b, int k) {
    if constexpr ((DBG & 4) != 0) return;
    // per-image buffer resources: 32-bit offsets, and a load past the range (the
    // a1 units >= XU, the dz2 slots >= 81) returns 0 without a branch
    if (k < 4) {
      const auto ra = make_rsrc(a1 + (size_t)b * 12800, 12800 * 4);
      const int off = tid + 512 * k < XU ? xsrc[k] * 4 : 0x7ffffff0;
      xs[k][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
      xs[k][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
    } else {
      const auto rd = make_rsrc(dz2 + (size_t)b * (81 * 64), 81 * 64 * 4);
      const int j = (k - 4) >> 1, e0 = 4 * ((k - 4) & 1), v = tid + 512 * j;
#pragma unroll
      for (int e = e0; e < e0 + 4; ++e) {
        const int r = 8 * (v >> 6) + e;
        const int off = v < DU && r < 81 ? (c2w_pix(r) * 64 + (v & 63)) * 4 : 0x7ffffff0;
        ds[j][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rd, off, 0, 0));
      }
    }
  };
  auto fetch = [&](int b) {
#pragma unroll
    for (int k = 0; k < 8; ++k) fetch_part(b, k);
  };
  auto put = [&](bool count) {   // count: add the dz2 to the bias partial
    if constexpr ((DBG & 2) != 0) return;
#pragma unroll
    for (int j = 0; j < XPER; ++j)
      if (tid + 512 * j < XU) {
        Frag3 f;
        split8(xs[j][0], xs[j][1], f, false);
        *reinterpret_cast<bf16x8*>(&X[xdst[j]]) = f.h;
        *reinterpret_cast<bf16x8*>(&X[XPL + xdst[j]]) = f.m;
        *reinterpret_cast<bf16x8*>(&X[2 * XPL + xdst[j]]) = f.l;
      }
#pragma unroll
    for (int j = 0; j < DPER; ++j) {
      const int v = tid + 512 * j;
      if (v < DU) {
        Frag3 f;
        split8(f32x4{ds[j][0], ds[j][1], ds[j][2], ds[j][3]}, f32x4{ds[j][4], ds[j][5], ds[j][6], ds[j][7]}, f,
               false);
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += count ? ds[j][e] : 0.f;
        const int off = (v & 63) * DR + 8 * (v >> 6);
        *reinterpret_cast<bf16x8*>(&D[off]) = f.h;
        *reinterpret_cast<bf16x8*>(&D[DPL + off]) = f.m;
        *reinterpret_cast<bf16x8*>(&D[2 * DPL + off]) = f.l;
      }
    }
  };
  f32x4 acc[4][4];   // [n tile j][co tile mt]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[j][mt] = zero4();
  const int Z = gridDim.x;
  int b = blockIdx.x;
  // the odd blocks start ~half an image late (s_sleep 100 = 6,400 clocks): every
  // block issues its next image's loads at the same k-steps, and in lock step the
  // whole chip's loads arrive as one burst per image (1.69 -> 1.61-1.63 ms, kbench)
  if ((DBG & 16) == 0 && (blockIdx.x & 1)) __builtin_amdgcn_s_sleep(100);
  if (b < B) {
    fetch(b);
    put(true);
  }
  __syncthreads();
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  for (; b < B; b += Z) {
    const bool pf = b + Z < B;
    const int bn = pf ? b + Z : b;   // the last image re-reads itself (no branch in the MFMA stream)
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
        if constexpr ((DBG & 8) != 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if ((3 * k) >> 1 == 4 * s + j) {
              fetch_part(bn, k);
              __builtin_amdgcn_sched_barrier(0);
            }
        } else if (4 * s + j < 8) {
          fetch_part(bn, 4 * s + j);
          __builtin_amdgcn_sched_barrier(0);   // the loads stay in their slot
        }
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
        if constexpr ((DBG & 1) == 0) {
          PPO_PRODUCTS(NP, PPO_PART)
        } else {   // keep the fragment reads live
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) acc[j][mt][0] += (float)a[mt].h[0] + (float)bf.h[0] + (float)bf.l[1];
        }
#undef PPO_PART
      }
    }
    __syncthreads();   // the image is consumed
    put(pf);   // unconditional: every load is waited for inside the iteration
    __syncthreads();   // the next image is in LDS
  }
  // this block's partial: C row 4g + r of co tile mt, column i16 of n tile j
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

// conv3 dgrad, image-resident on the bf16 matrix cores (exact split, DESIGN.md
// §3): dz2[m][ci] = [a2 > 0] Σ_(ky,kx,co) dz3[y-ky][x-kx][co] W3d[ci][(ky,kx,co)],
// m = (y, x) over the 9 x 9 input (81 rows in 6 tiles of 16), k-step = tap, lane
// group g = co chunk.  One persistent block (8 waves) per CU walks images; per
// image the LDS holds dz3 split into three bf16 planes on a zero-padded grid of
// width 25 (dz3 pixel (oy, ox) at (oy + 2) * 25 + ox + 2; 11 rows), in 16-B units
// c * 288 + pixel: row m's tap pixel is 25 y + x + const ≡ m + const (mod 16), so
// the 16 rows of a tile hit distinct slots (conflict-free ds_read_b128), and out-of-
// range taps read zeros.  Two stages (2 x 55,296 B) plus the a2 ReLU mask as
// bytes (2 x 5,184 B): the next image is staged before the compute, one barrier
// per image.  Wave w: ci tile w & 3 (weights, 9 taps x 3 planes, in 108 VGPRs),
// row tiles 3 (w >> 2) .. +2.
// BITS: the a2 ReLU mask comes as bits (a2 points at u64 words [B][81] from
// ppo_conv2_fwd_mask: 648 B instead of 20.7 KB per image).
template <int NP, bool BITS = false>
__global__ __launch_bounds__(512) void conv3_dgrad_x9_kernel(const float* __restrict__ dz3, int B,
                                                            const uint16_t* __restrict__ wpl,
                                                            const float* __restrict__ a2,
                                                            float* __restrict__ dz2, int stagger) {
  constexpr int GW = 25, CS = 288, PLU = 4 * CS, KS = 9, WN = 64 * 288;
  constexpr int DU = 49 * 4, MC = 81 * 64 / 4, MPER = (MC + 511) / 512;
  __shared__ __attribute__((aligned(16))) uint16_t S[2][3 * PLU * 8];
  __shared__ __attribute__((aligned(16))) uint32_t Mk[2][MC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int nt = wave & 3, mh = wave >> 2, ci = 16 * nt + i16;
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + ci * 288 + 32 * s + 8 * g);
  wait_vm0();
  for (int i = tid; i < 2 * 3 * PLU; i += 512) reinterpret_cast<uint4*>(&S[0][0])[i] = uint4{0, 0, 0, 0};
  // unit index of this lane's A fragment per row tile for tap (0, 0); tap
  // (ky, kx) subtracts 25 ky + kx
  // Row tiles and the taps they need: a tap whose source pixel is off the 7 x 7
  // grid for all 16 rows of a tile is skipped (tile 0: ky <= 1, tile 4: ky >= 1,
  // tile 5 = pixel 80 alone: tap (2, 2) only) — 40 of the 54 tile-taps.  Wave
  // halves take tiles {1, 2, 5} (19 tile-taps) and {0, 3, 4} (21).
  constexpr unsigned TILES = 0x430521u;   // nibbles: tiles of half 0 (1, 2, 5), half 1 (0, 3, 4)
  // tap masks per tile (bit 3 ky + kx): {0x03F, 0x1FF, 0x1FF, 0x1FF, 0x1F8, 0x100}
  int qrow[3], tl[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    tl[t] = (TILES >> (4 * (3 * mh + t))) & 15;
    const int m = min(16 * tl[t] + i16, 80), y = m / 9, x = m - 9 * y;   // dummy rows: pixel 80
    qrow[t] = g * CS + (y + 2) * GW + x + 2;
  }
  f32x4 stg[2];
  f32x4 mst[BITS ? 1 : MPER];
  uint2 mbv;
  auto fetch = [&](int b) {
    if (tid < DU) {
      const f32x4* src = reinterpret_cast<const f32x4*>(dz3 + (size_t)b * 1568);
      stg[0] = src[2 * tid];
      stg[1] = src[2 * tid + 1];
    }
    if constexpr (BITS) {
      if (tid < 81) mbv = reinterpret_cast<const uint2*>(a2)[(size_t)b * 81 + tid];
    } else {
      const f32x4* ms = reinterpret_cast<const f32x4*>(a2 + (size_t)b * 5184);
#pragma unroll
      for (int j = 0; j < MPER; ++j)
        if (tid + 512 * j < MC) mst[j] = ms[tid + 512 * j];
    }
  };
  auto put = [&](int buf) {
    if (tid < DU) {   // unit tid: dz3 pixel tid >> 2, co chunk tid & 3
      const int px = tid >> 2, oy = px / 7, ox = px - 7 * oy;
      const int q = (tid & 3) * CS + (oy + 2) * GW + ox + 2;
      Frag3 f;
      split8(stg[0], stg[1], f, false);
      *reinterpret_cast<bf16x8*>(&S[buf][8 * q]) = f.h;
      *reinterpret_cast<bf16x8*>(&S[buf][8 * (PLU + q)]) = f.m;
      *reinterpret_cast<bf16x8*>(&S[buf][8 * (2 * PLU + q)]) = f.l;
    }
    if constexpr (BITS) {
      if (tid < 81) reinterpret_cast<uint2*>(Mk[buf])[tid] = mbv;
    } else {
#pragma unroll
      for (int j = 0; j < MPER; ++j) {
        const int c = tid + 512 * j;
        if (c < MC)
          Mk[buf][c] = (mst[j][0] > 0.f ? 1u : 0u) | (mst[j][1] > 0.f ? 0x100u : 0u) |
                       (mst[j][2] > 0.f ? 0x10000u : 0u) | (mst[j][3] > 0.f ? 0x1000000u : 0u);
      }
    }
  };
  __syncthreads();   // the zeroed pads
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
    put(0);
    if (b + G < B) fetch(b + G);
  }
  __syncthreads();
  // stagger: waves 4-7 (the second wave of every SIMD) stage the next image
  // after their compute instead of before it, so each SIMD's matrix pipe has
  // one computing wave while the other splits and stores
  const bool late = stagger && wave >= 4;
  for (; b < B; b += G) {
    if (!late) {
      if (b + G < B) put(cur ^ 1);
      if (b + 2 * G < B) fetch(b + 2 * G);
    }
    const uint16_t* Sc = S[cur];
    f32x4 acc[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) acc[t] = zero4();
    // the tap masks are compile-time in each of the two instantiations, so the
    // skipped (tile, tap) pairs vanish from the unrolled schedule
    auto compute = [&](auto M0, auto M1, auto M2) {
      constexpr unsigned msk[3] = {decltype(M0)::value, decltype(M1)::value, decltype(M2)::value};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int toff = -(GW * (s / 3) + s % 3);
        const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
        Frag3 a[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          if (!((msk[u] >> s) & 1u)) continue;
          const uint16_t* q = Sc + 8 * (qrow[u] + toff);
          a[u].h = *reinterpret_cast<const bf16x8*>(q);
          a[u].m = *reinterpret_cast<const bf16x8*>(q + 8 * PLU);
          a[u].l = *reinterpret_cast<const bf16x8*>(q + 16 * PLU);
        }
#define PPO_PART(X, Y) \
  _Pragma("unroll") for (int u = 0; u < 3; ++u) if ((msk[u] >> s) & 1u) acc[u] = mma(w.Y, a[u].X, acc[u]);
        PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
      }
    };
    using std::integral_constant;
    if (mh == 0)
      compute(integral_constant<unsigned, 0x1FF>{}, integral_constant<unsigned, 0x1FF>{},
              integral_constant<unsigned, 0x100>{});
    else
      compute(integral_constant<unsigned, 0x03F>{}, integral_constant<unsigned, 0x1FF>{},
              integral_constant<unsigned, 0x1F8>{});
    // epilogue: C row 4g + r of tile t is input pixel m; ReLU mask of a2
    // swapped orientation (weights as the MFMA A operand): lane (i16, g) holds
    // pixel 16 tl + i16, channels c0 = 16 nt + 4g .. +3 — one 16-B store per tile
    const uint8_t* mk = reinterpret_cast<const uint8_t*>(Mk[cur]);
    const auto rs = make_rsrc(dz2 + (size_t)b * 5184, 5184 * 4);
    const int c0 = 16 * nt + 4 * g;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int m = 16 * tl[t] + i16, mm = min(m, 80);
      const uint32_t mw = Mk[cur][2 * mm + (c0 >> 5)] >> (c0 & 31);
      f32x4 y;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool keep = BITS ? ((mw >> r) & 1u) != 0 : mk[mm * 64 + c0 + r] != 0;
        y[r] = keep ? acc[t][r] : 0.f;
      }
      bstore_f32x4(y, rs, m < 81 ? 4 * (m * 64 + c0) : -1);
    }
    if (late) {
      if (b + G < B) put(cur ^ 1);
      if (b + 2 * G < B) fetch(b + 2 * G);
    }
    __syncthreads();   // every wave is done with stage cur; stage cur ^ 1 is complete
    cur ^= 1;
  }
}

// conv3 forward, image-resident on the bf16 matrix cores (exact split, DESIGN.md
// §3): a3[b][(oy, ox)][co] = relu(b3[co] + Σ_(ky,kx,ci) a2[oy+ky][ox+kx][ci] W3p[co][k]).
// GEMM rows run over the 9-wide input grid, m = 9 oy + ox (ox = 7, 8 dummy: 63 rows
// in 4 tiles, as many as the 49 real rows need), so row m's tap pixel is m + 9 ky
// + kx — 16 consecutive pixels per tile, conflict-free ds_read_b128 with chunk c of
// pixel p at c ^ ((p >> 1) & 7) (128-B pixel rows).  k-step = (tap, ci half), lane
// group g = 8-ci chunk.  Per image the LDS holds a2 split into three bf16 planes
// (84 pixel rows, the last 3 zero, reached by dummy rows only): 2 stages x 32,256 B,
// the next image staged before the compute.  Wave w: co tile w & 1, K half
// (w >> 1) & 1 (taps 0-4.5 / 4.5-8: 9 k-steps, weights in 108 VGPRs), row tiles
// 2 (w >> 2) .. +1; K half 1 hands its partial sums over through LDS.
constexpr int C3F_PL = 84 * 64;   // conv3 forward: bf16 per plane
constexpr int C3F_LDS = 2 * 3 * C3F_PL * 2 + 2 * 2 * 2 * 2 * 64 * 16;   // stages + K-half partials (80,896 B)
template <int NP>
__device__ __forceinline__ void conv3_fwd_x9_body(const float* __restrict__ a2, int B,
                                                  const uint16_t* __restrict__ wpl, const float* __restrict__ bias,
                                                  float* __restrict__ out, uint8_t* __restrict__ lds) {
  constexpr int NPX = 84, PL = NPX * 64, KS = 9, WN = 32 * 576, UNITS = 81 * 8, UPER = (UNITS + 511) / 512;
  static_assert(PL == C3F_PL, "plane size");
  uint16_t (*const S)[3 * PL] = reinterpret_cast<uint16_t (*)[3 * PL]>(lds);
  f32x4 (*const R)[2][2][2][64] = reinterpret_cast<f32x4 (*)[2][2][2][64]>(lds + 2 * 3 * PL * 2);   // [stage][co tile][row half][tile][lane]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int nt = wave & 1, kh = (wave >> 1) & 1, mh = wave >> 2, co = 16 * nt + i16;
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + co * 576 + (9 * kh + s) * 32 + 8 * g);
  // swapped orientation (weights as the MFMA A operand): lane (i16, g) holds
  // row 16 t + i16, channels 16 nt + 4g .. +3 — one 16-B store per tile
  const f32x4 bv4 = *reinterpret_cast<const f32x4*>(bias + 16 * nt + 4 * g);
  wait_vm0();
  for (int i = tid; i < 2 * 3 * PL / 8; i += 512) reinterpret_cast<uint4*>(&S[0][0])[i] = uint4{0, 0, 0, 0};
  f32x4 stg[UPER][2];
  // unit j of image b through a per-image buffer resource (units past the image
  // read out of range: 0, no branch)
  auto fetch_unit = [&](int b, int j) {
    const auto ra = make_rsrc(a2 + (size_t)b * 5184, 5184 * 4);
    const int u = tid + 512 * j, off = u < UNITS ? 32 * u : 0x7fffffe0;
    stg[j][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
    stg[j][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
  };
  auto fetch = [&](int b) {
#pragma unroll
    for (int j = 0; j < UPER; ++j) fetch_unit(b, j);
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int j = 0; j < UPER; ++j) {
      const int u = tid + 512 * j;
      if (u < UNITS) {
        const int p = u >> 3, off = p * 64 + 8 * ((u & 7) ^ ((p >> 1) & 7));
        Frag3 f;
        split8(stg[j][0], stg[j][1], f, false);
        *reinterpret_cast<bf16x8*>(&S[buf][off]) = f.h;
        *reinterpret_cast<bf16x8*>(&S[buf][PL + off]) = f.m;
        *reinterpret_cast<bf16x8*>(&S[buf][2 * PL + off]) = f.l;
      }
    }
  };
  __syncthreads();   // the zeroed pad rows
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
    put(0);
    fetch(b + G < B ? b + G : b);
  }
  __syncthreads();
  for (; b < B; b += G) {
    // the stage write unconditional (past the end: a copy of this image into the
    // idle stage), the image after next fetched one unit per k-step 1, 3 inside the
    // MFMA stream instead of in a burst here
    put(cur ^ 1);
    const int bnn = b + 2 * G < B ? b + 2 * G : b;
    const uint16_t* Sc = S[cur];
    f32x4 acc[2] = {zero4(), zero4()};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int ks = 9 * kh + s, tap = ks >> 1, ky = tap / 3, kx = tap - 3 * ky, c = 4 * (ks & 1) + g;
      const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
      Frag3 a[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int p = 16 * (2 * mh + u) + i16 + 9 * ky + kx;
        const uint16_t* q = Sc + p * 64 + 8 * (c ^ ((p >> 1) & 7));
        a[u].h = *reinterpret_cast<const bf16x8*>(q);
        a[u].m = *reinterpret_cast<const bf16x8*>(q + PL);
        a[u].l = *reinterpret_cast<const bf16x8*>(q + 2 * PL);
      }
#define PPO_PART(X, Y) \
  _Pragma("unroll") for (int u = 0; u < 2; ++u) acc[u] = mma(w.Y, a[u].X, acc[u]);
      PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
      if (s == 1 || s == 3) {
        fetch_unit(bnn, s >> 1);
        __builtin_amdgcn_sched_barrier(0);   // the loads stay in their slot
      }
    }
    if (kh == 1) {
      R[cur][nt][mh][0][lane] = acc[0];
      R[cur][nt][mh][1][lane] = acc[1];
    }
    __syncthreads();   // stage cur consumed, stage cur ^ 1 complete, partials in R[cur]
    if (kh == 0) {
      const auto rs = make_rsrc(out + (size_t)b * (49 * 32), 49 * 32 * 4);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f32x4 v = acc[u] + R[cur][nt][mh][u][lane];
        const int m = 16 * (2 * mh + u) + i16, oy = m / 9, ox = m - 9 * oy;
        f32x4 y;
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + bv4[r], 0.f);
        bstore_f32x4(y, rs, (ox < 7 && oy < 7) ? 4 * ((7 * oy + ox) * 32 + 16 * nt + 4 * g) : -1);
      }
    }
    cur ^= 1;
  }
}

template <int NP>
__global__ __launch_bounds__(512) void conv3_fwd_x9_kernel(const float* __restrict__ a2, int B,
                                                          const uint16_t* __restrict__ wpl,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out, int stagger) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[C3F_LDS];
  (void)stagger;
  conv3_fwd_x9_body<NP>(a2, B, wpl, bias, out, lds);
}

// conv3 forward with compact rows (round 5; the row -> output map c3_row_q since round 6,
// the original order is described below): GEMM row m = 7 oy + ox over the 49 real
// outputs (the 9-wide grid above issues 64 rows for them), row tiles 0-2 (m < 48)
// and output 48 = (6, 6) left to conv3_lone_tiles.  Wave w: co tile w & 1, K half
// (w >> 1) & 1; with NT = 768 threads (the standalone launch, 3 waves per SIMD) row
// tile w >> 2, with NT = 512 (the fused trunk's third phase) row tiles 0-1 for waves
// 0-3 and tile 2 for waves 4-7 — waves w and w + 4 share a SIMD, so the SIMD's
// matrix core runs 3 tiles per image instead of the 9-wide grid's 4.  A lane's tap
// pixel is p0(m) + 9 ky + kx, p0 = 9 oy + ox (a per-lane base: the 16 rows of a tile
// are no longer 16 consecutive pixels, so some ds_read_b128 groups meet 2-way bank
// conflicts).  The same operand splits, k-steps, part order and K-half sum as
// conv3_fwd_x9_body, so every output is bit-identical to it whatever the wave count.
// LONE: the lone output of the block's own images after its image loop (round 6,
// VERDICT r05 item 7); else conv3_fwd_lone_kernel covers it (C3F_COMPACT = 1).
constexpr int C3L_IR = 73;    // 16-B units per staged lone patch and plane (72 + pad)
constexpr int C3L_PL = 16 * C3L_IR;
constexpr int C3L_LDS = 2 * 3 * C3L_PL * 16 + 2 * 64 * 16;   // two 3-plane patch stages + K-half partials (114,176 B)
constexpr int C3C_LDS0 = 2 * 3 * 84 * 80 * 2 + 2 * 2 * 3 * 64 * 16;   // the image loop: stages + K-half partials (92,928 B)
constexpr int C3C_LDS = C3C_LDS0 > C3L_LDS ? C3C_LDS0 : C3L_LDS;   // the lone tiles after it reuse the LDS

// Compact rows of conv3's forward (round 6): tile row 16 t + r computes output pixel
// q = c3_row_q[16 t + r] (q = 7 oy + ox), the 49th, (6, 0), is the lone output.  With
// 160-B pixel rows (16-B slot 10 p + c of input pixel p = 9 oy + ox + tap, chunk c) the
// 16 lanes of a ds_read_b128 group — rows {0-3, 12-15} at chunk c0 and rows {4-11} at
// c0 + 1, or the reverse — hit distinct slots for every tap iff each of those two row
// sets covers the 8 residues p mod 8 once: this table does that for all 3 tiles (the
// residue of (6, 6) would have left one set a duplicate, hence the lone (6, 0)); the
// oy-major order before it met 2-way conflicts in most groups (tools/conv3_bank_model.py)
constexpr int C3_LONE_Y = 6, C3_LONE_X = 0, C3_LONE_Q = 7 * C3_LONE_Y + C3_LONE_X;
__constant__ uint8_t c3_row_q[48] = {0,  1,  2,  3,  20, 7,  8,  9,  10, 11, 12, 19, 4,  5,  6,  13,
                                     26, 27, 14, 15, 32, 33, 34, 21, 22, 23, 24, 31, 16, 17, 18, 25,
                                     38, 39, 40, 41, 44, 45, 46, 47, 48, 35, 36, 43, 28, 29, 30, 37};

// ReLU mask bits of conv3's output (the training forward; read by the fc dgrad instead
// of the 411 MB fp32 activation): uint16 [B][49 pixels][2 channel tiles], bit j of word
// (p, t) = output channel 16 t + j of pixel p > 0.  Lane (g, i16) holds channels
// 16 t + 4 g + r (r < 4) of one pixel; lanes i16, i16 + 16, +32, +48 combine by two
// shuffles and lane g = 0 stores the word.
__device__ __forceinline__ void conv3_mask_store(const f32x4& y, int g, uint16_t* dst) {
  uint32_t w = ((y[0] > 0.f ? 1u : 0u) | (y[1] > 0.f ? 2u : 0u) | (y[2] > 0.f ? 4u : 0u) | (y[3] > 0.f ? 8u : 0u))
               << (4 * g);
  w |= (uint32_t)__shfl_xor((int)w, 16, 64);
  w |= (uint32_t)__shfl_xor((int)w, 32, 64);
  if (g == 0) *dst = (uint16_t)w;
}

// conv3 forward of output 48 = (6, 6) for 16 images per tile: tiles t0, t0 + tstep, ...
// of the images base + stride * i (i < nimg; row i16 of the B operand is image base +
// stride * (16 t + i16)); the same operands, MFMA sequence, K-half sum and epilogue as
// the compact kernel (bit-identical).  Waves 0-3 compute (co tile w & 1, K half w >> 1,
// their weight fragments bw), every thread of the NT stages.  As conv2's lone tiles,
// the tile's 16 patches (3 rows of 3 pixels x 64 channels, 768 contiguous bytes per
// row) are loaded once per block, the next tile's in registers during this tile's
// MFMAs, and staged in LDS (two stages, image rows padded by 16 B).
template <int NP, int NT>
__device__ __forceinline__ void conv3_lone_tiles(const float* __restrict__ a2, const bf16x8 (&bw)[9][3],
                                                 const float* __restrict__ bias, float* __restrict__ out,
                                                 uint8_t* __restrict__ lds, long long base, long long stride,
                                                 int nimg, int t0, int tstep, uint16_t* __restrict__ m3 = nullptr) {
  constexpr int KS = 9, M = C3_LONE_Q, IR = C3L_IR, PL = C3L_PL, NCH = 16 * 72, NPC = (NCH + NT - 1) / NT;
  uint4 (*const P)[3 * PL] = reinterpret_cast<uint4 (*)[3 * PL]>(lds);
  f32x4* const R = reinterpret_cast<f32x4*>(lds + 2 * 3 * PL * 16);
  const int tid = threadIdx.x, lane = tid & 63, i16 = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = wave & 1, kh = (wave >> 1) & 1;
  const int ntile = (nimg + 15) / 16;
  // chunk c = tid + NT j: image c / 72, 8-channel chunk u = c % 72 of its patch = tap
  // (3 ky + kx) * 8 + channel octet; a2 offset ((LY + ky) * 9 + LX) * 64 + (u % 24) * 8 for
  // the lone output (LY, LX) = (C3_LONE_Y, C3_LONE_X).
  // Round 6: split into the bf16 planes once here, not by each computing wave at
  // fragment read (as conv2_lone_tiles)
  f32x4 pc[NPC][2];
  auto fetch = [&](int T) {   // past the last tile / image: zeros, nothing loaded
#pragma unroll
    for (int j = 0; j < NPC; ++j) {
      const int c = tid + NT * j, im = c / 72, u = c - 72 * im, ky = u / 24, i = 16 * T + im;
      const bool live = c < NCH && T < ntile && i < nimg;
      const float* src = a2 + (size_t)(base + stride * (live ? i : 0)) * 5184 + ((C3_LONE_Y + ky) * 9 + C3_LONE_X) * 64 +
                         (u - 24 * ky) * 8;
      pc[j][0] = live ? *reinterpret_cast<const f32x4*>(src) : zero4();
      pc[j][1] = live ? *reinterpret_cast<const f32x4*>(src + 4) : zero4();
    }
  };
  auto put = [&](int st) {
#pragma unroll
    for (int j = 0; j < NPC; ++j) {
      const int c = tid + NT * j, im = c / 72;
      if (c < NCH) {
        const int o = im * IR + (c - 72 * im);
        Frag3 f;
        split8(pc[j][0], pc[j][1], f, false);
        P[st][o] = __builtin_bit_cast(uint4, f.h);
        P[st][PL + o] = __builtin_bit_cast(uint4, f.m);
        P[st][2 * PL + o] = __builtin_bit_cast(uint4, f.l);
      }
    }
  };
  fetch(t0);
  put(0);
  __syncthreads();
  int cur = 0;
  for (int T = t0; T < ntile; T += tstep) {
    fetch(T + tstep);
    const int i = 16 * T + i16;
    const long long b = base + stride * (long long)i;
    f32x4 acc = zero4();
    if (wave < 4) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int ks = 9 * kh + s, tap = ks >> 1, c = 4 * (ks & 1) + g, o = i16 * IR + tap * 8 + c;
        Frag3 a;
        a.h = __builtin_bit_cast(bf16x8, P[cur][o]);
        a.m = __builtin_bit_cast(bf16x8, P[cur][PL + o]);
        a.l = __builtin_bit_cast(bf16x8, P[cur][2 * PL + o]);
        const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
#define PPO_PART(X, Y) acc = mma(w.Y, a.X, acc);
        PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
      }
      if (kh == 1) R[nt * 64 + lane] = acc;
    }
    put(cur ^ 1);   // the stage read one tile ago (the last barrier retired its reads)
    __syncthreads();   // partials in R; stage cur ^ 1 complete
    if (wave < 2 && i < nimg) {   // kh == 0
      const f32x4 bv4 = *reinterpret_cast<const f32x4*>(bias + 16 * nt + 4 * g);
      const f32x4 v = acc + R[nt * 64 + lane];
      f32x4 y;
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + bv4[r], 0.f);
      *reinterpret_cast<f32x4*>(out + (size_t)b * (49 * 32) + M * 32 + 16 * nt + 4 * g) = y;
      // the four lanes of image i (g = 0..3) share its activity: the shuffles read live lanes
      if (m3) conv3_mask_store(y, g, m3 + (size_t)b * 98 + M * 2 + nt);
    }
    __syncthreads();   // R read before the next tile's partials
    cur ^= 1;
  }
}

template <int NP, int NT, bool LONE>
__device__ __forceinline__ void conv3_fwd_c3_body(const float* __restrict__ a2, int B,
                                                  const uint16_t* __restrict__ wpl, const float* __restrict__ bias,
                                                  float* __restrict__ out, uint8_t* __restrict__ lds,
                                                  uint16_t* __restrict__ m3 = nullptr) {
  static_assert(NT == 512 || NT == 768, "8 or 12 waves");
  // pixel rows of 80 bf16 (160 B, 16-B chunk c of pixel p at 16-B slot 10 p + c): round 6,
  // for the compact rows' tap reads, whose 16 lanes of a ds_read_b128 group are 16
  // pixels 9 oy + ox + tap apart: 2-way bank conflicts at most, against up to 3-way with
  // 128-B rows and the chunk swizzle c ^ ((p >> 1) & 7) (55 % of the LDS-active cycles
  // conflicted, profiles/r06_s19_conv_fwd_sq.json; tools-free model in DESIGN §A.0)
  constexpr int NPX = 84, PR = 80, PL = NPX * PR, KS = 9, WN = 32 * 576, UNITS = 81 * 8,
                UPER = (UNITS + NT - 1) / NT;
  uint16_t (*const S)[3 * PL] = reinterpret_cast<uint16_t (*)[3 * PL]>(lds);
  f32x4 (*const R)[2][3][64] = reinterpret_cast<f32x4 (*)[2][3][64]>(lds + 2 * 3 * PL * 2);   // [stage][co tile][row tile][lane]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int nt = wave & 1, kh = (wave >> 1) & 1, co = 16 * nt + i16;
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + co * 576 + (9 * kh + s) * 32 + 8 * g);
  const f32x4 bv4 = *reinterpret_cast<const f32x4*>(bias + 16 * nt + 4 * g);
  wait_vm0();
  for (int i = tid; i < 2 * 3 * PL / 8; i += NT) reinterpret_cast<uint4*>(&S[0][0])[i] = uint4{0, 0, 0, 0};
  f32x4 stg[UPER][2];
  auto fetch = [&](int b) {   // a per-image buffer resource: units past the image read 0, no branch
    const auto ra = make_rsrc(a2 + (size_t)b * 5184, 5184 * 4);
#pragma unroll
    for (int j = 0; j < UPER; ++j) {
      const int u = tid + NT * j, off = u < UNITS ? 32 * u : 0x7fffffe0;
      stg[j][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
      stg[j][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
    }
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int j = 0; j < UPER; ++j) {
      const int u = tid + NT * j;
      if (u < UNITS) {
        const int p = u >> 3, off = p * PR + 8 * (u & 7);
        Frag3 f;
        split8(stg[j][0], stg[j][1], f, false);
        *reinterpret_cast<bf16x8*>(&S[buf][off]) = f.h;
        *reinterpret_cast<bf16x8*>(&S[buf][PL + off]) = f.m;
        *reinterpret_cast<bf16x8*>(&S[buf][2 * PL + off]) = f.l;
      }
    }
  };
  __syncthreads();   // the zeroed pad rows
  const int G = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
    put(0);
    fetch(b + G < B ? b + G : b);
  }
  __syncthreads();
  // row tiles of this wave: mt0 .. mt0 + ntl - 1; the k loop takes the count as a
  // compile-time constant (a run-time bound would issue the second tile's MFMAs on
  // every wave), the barriers stay outside the wave-dependent branch
  const int mt0 = NT == 768 ? (wave >> 2) : (wave < 4 ? 0 : 2);
  const int ntl = NT == 768 || wave >= 4 ? 1 : 2;
  int p0[2], q0[2];   // tap-(0, 0) input pixel and output pixel of this lane's row per tile
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int q = c3_row_q[mt0 + t < 3 ? 16 * (mt0 + t) + i16 : 0], oy = q / 7;   // (no tile 3: unused)
    q0[t] = q;
    p0[t] = 9 * oy + (q - 7 * oy);
  }
  for (; b < B; b += G) {
    put(cur ^ 1);   // unconditional (past the end: a copy of this image into the idle stage)
    const int bnn = b + 2 * G < B ? b + 2 * G : b;
    const uint16_t* Sc = S[cur];
    f32x4 acc[2] = {zero4(), zero4()};
    auto kloop = [&](auto ntc) __attribute__((always_inline)) {
      constexpr int NTL = decltype(ntc)::value;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int ks = 9 * kh + s, tap = ks >> 1, ky = tap / 3, kx = tap - 3 * ky, c = 4 * (ks & 1) + g;
        const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
        Frag3 a[NTL];
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
          const int p = p0[t] + 9 * ky + kx;
          const uint16_t* q = Sc + p * PR + 8 * c;
          a[t].h = *reinterpret_cast<const bf16x8*>(q);
          a[t].m = *reinterpret_cast<const bf16x8*>(q + PL);
          a[t].l = *reinterpret_cast<const bf16x8*>(q + 2 * PL);
        }
#define PPO_PART(X, Y) \
  _Pragma("unroll") for (int t = 0; t < NTL; ++t) acc[t] = mma(w.Y, a[t].X, acc[t]);
        PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
        if (s == 1) {
          fetch(bnn);
          __builtin_amdgcn_sched_barrier(0);   // the loads stay in their slot
        }
      }
    };
    if constexpr (NT == 768) kloop(std::integral_constant<int, 1>{});
    else if (wave < 4) kloop(std::integral_constant<int, 2>{});
    else kloop(std::integral_constant<int, 1>{});
    if (kh == 1) {
      R[cur][nt][mt0][lane] = acc[0];
      if (ntl == 2) R[cur][nt][mt0 + 1][lane] = acc[1];
    }
    __syncthreads();   // stage cur consumed, stage cur ^ 1 complete, partials in R[cur]
    if (kh == 0) {
      const auto rs = make_rsrc(out + (size_t)b * (49 * 32), 49 * 32 * 4);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t < ntl) {
          const f32x4 v = acc[t] + R[cur][nt][mt0 + t][lane];
          f32x4 y;
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + bv4[r], 0.f);
          bstore_f32x4(y, rs, 4 * (q0[t] * 32 + 16 * nt + 4 * g));
          if (m3) conv3_mask_store(y, g, m3 + (size_t)b * 98 + q0[t] * 2 + nt);
        }
      }
    }
    cur ^= 1;
  }
  if constexpr (LONE) {
    __syncthreads();   // the last image's partials (R) are read
    const int blk = blockIdx.x;
    const int nimg = blk < B ? (B - 1 - blk) / G + 1 : 0;
    conv3_lone_tiles<NP, NT>(a2, bw, bias, out, lds, blk, G, nimg, 0, 1, m3);
  }
}

#ifndef C3F_COMPACT
#define C3F_COMPACT 2   // standalone conv3 forward: 2 compact rows + the lone output in the same
                        // launch (default), 1 compact rows + conv3_fwd_lone_kernel, 0 the 9-wide grid
#endif
template <int NP>
__global__ __launch_bounds__(768) void conv3_fwd_c3_kernel(const float* __restrict__ a2, int B,
                                                           const uint16_t* __restrict__ wpl,
                                                           const float* __restrict__ bias,
                                                           float* __restrict__ out, uint16_t* __restrict__ m3) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[C3C_LDS];
  conv3_fwd_c3_body<NP, 768, C3F_COMPACT == 2>(a2, B, wpl, bias, out, lds, m3);
}

template <int NP>
__global__ __launch_bounds__(256) void conv3_fwd_lone_kernel(const float* __restrict__ a2, int B,
                                                             const uint16_t* __restrict__ wpl,
                                                             const float* __restrict__ bias,
                                                             float* __restrict__ out) {
  constexpr int KS = 9, WN = 32 * 576;
  __shared__ __attribute__((aligned(16))) uint8_t lds[C3L_LDS];
  const int tid = threadIdx.x, i16 = tid & 15, g = (tid & 63) >> 4, wave = tid >> 6;
  const int co = 16 * (wave & 1) + i16, kh = wave >> 1;
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + co * 576 + (9 * kh + s) * 32 + 8 * g);
  conv3_lone_tiles<NP, 256>(a2, bw, bias, out, lds, 0, 1, B, blockIdx.x, gridDim.x);
}

// The rollout's CNN trunk in one launch: conv1 -> conv2 -> conv3 forward as three
// phases of one persistent grid (one block per CU).  Every phase maps image b to
// block b mod G, so a block consumes only its own outputs of the phase before:
// no grid-wide synchronisation, only each wave's stores retired (vmcnt) and a
// block barrier between phases, then an agent-scope acquire (L1 invalidate).
// This removes the two kernel boundaries inside the trunk — 10.3-10.4 us each
// between these persistent kernels at the rollout's 4,096 images (c5 kernel trace,
// profiles/r05_l_c5_kernel_stats.csv) — and each phase is the unchanged kernel body
// (bit-identical outputs to the three launches).  The phases share one LDS buffer
// (the largest phase, conv2: 154,368 B).
constexpr int TRUNK_LDS = C2F_LDS > C3F_LDS ? (C2F_LDS > 2 * 4 * C1S * 2 ? C2F_LDS : 2 * 4 * C1S * 2)
                                            : (C3F_LDS > 2 * 4 * C1S * 2 ? C3F_LDS : 2 * 4 * C1S * 2);
static_assert(C3L_LDS <= TRUNK_LDS && C3C_LDS0 <= TRUNK_LDS, "the trunk's conv3 phase in the shared LDS");
__device__ __forceinline__ void trunk_phase_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's output stores are in L2
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // no stale L1 line under the next phase's loads
}
template <int NP, bool MASK>
__global__ __launch_bounds__(512) void trunk_fwd_kernel(const uint8_t* __restrict__ obs, const int64_t* __restrict__ idx,
                                                       long long row0, int B, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, float* __restrict__ a1,
                                                       uint16_t* __restrict__ m1, const uint16_t* __restrict__ w2pl,
                                                       const float* __restrict__ b2, float* __restrict__ a2,
                                                       uint16_t* __restrict__ m2, const uint16_t* __restrict__ w3pl,
                                                       const float* __restrict__ b3, float* __restrict__ a3) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[TRUNK_LDS];
  conv1_fwd_bf16x3_body<4, MASK, NP == 1 ? 1 : 3>(obs, idx, row0, B, w1, b1, a1, m1,
                                                   reinterpret_cast<uint16_t (*)[4 * C1S]>(lds));
  trunk_phase_sync();
  conv2_fwd_x9c_body<NP, MASK, 0, 5, true>(a1, B, w2pl, b2, a2, m2, lds);
  trunk_phase_sync();
  conv3_fwd_c3_body<NP, 512, true>(a2, B, w3pl, b3, a3, lds);
}

// conv3 weight gradient, image-resident on the bf16 matrix cores (exact split,
// DESIGN.md §3): dW3[co][k] = Σ_pixels dz3[m][co] · a2[oy+ky][ox+kx][ci], k = (ky,
// kx, ci); per image a 32 x 576 x 49 product, accumulated in registers over the
// block's images and written once as its split-K partial (slab [Z][32][576],
// bias partials [Z][32]).  Reduction slot r = 8 oy + ox (ox = 7 and oy = 7 are
// dummy slots, dz = 0): 64 slots = 2 k-steps.  Per image (2 stages) the LDS holds
//   X [3][9 x 12 px][64 ci]  a2 split into bf16 planes, pixel P = 12 y + x, 128-B
//                            rows; the B fragment (8 slots x 16 ci of one tap) is two
//                            ds_read_b64_tr_b16 per plane whose 4-slot row groups
//                            are 4 consecutive ox and the next oy (P + 12): with
//                            8-B unit u of pixel P at u ^ 4 ((P >> 1) & 3) every
//                            32-lane half hits distinct banks
//   D [3][32 co][112]        dz3 transposed to [co][slot] (224-B rows: conflict-free
//                            ds_read_b128 A fragments)
// 12 waves (3 per SIMD), wave w: n tiles 3w .. 3w+2 (both co tiles).
template <int NP>
__global__ __launch_bounds__(768) void conv3_wgrad_x9_kernel(const float* __restrict__ dz3,
                                                            const float* __restrict__ a2, int B,
                                                            float* __restrict__ slab,
                                                            float* __restrict__ slab_bias) {
  constexpr int NT = 768, XPL = 108 * 64, DR = 112, DPL = 32 * DR;
  constexpr int XU = 81 * 8, XPER = (XU + NT - 1) / NT, DU = 32 * 8;
  __shared__ __attribute__((aligned(16))) uint16_t X[2][3 * XPL];
  __shared__ __attribute__((aligned(16))) uint16_t D[2][3 * DPL];
  __shared__ float bred[DU];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int q = i16 >> 2, p = i16 & 3;
  // tap-(0,0) pixel of the row this lane addresses in the tr reads of k-step s,
  // half h (dummy slots read pixel (6, 6): finite, times dz = 0)
  int Pb[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 32 * s + 8 * g + 4 * h + q;
      int oy = r >> 3, ox = r & 7;
      if (oy > 6 || ox > 6) { oy = 6; ox = 6; }
      Pb[s][h] = 12 * oy + ox;
    }
  f32x4 xs[XPER][2];
  float ds[7];
  float bsum = 0.f;   // bias partial of co = tid & 31 (threads < 256: slots of row oy = tid >> 5)
  // the next image's loads in two parts (a2 units; dz3 slots), issued inside the
  // MFMA stream of k-step 0 (as conv2's weight gradient), through per-image buffer
  // resources: lanes past the units / the 7 dz rows read out of range (0), no branch
  static_assert(XPER == 1, "one a2 unit per thread");
  auto fetch_part = [&](int b, int part) {
    if (part == 0) {
      const auto ra = make_rsrc(a2 + (size_t)b * 5184, 5184 * 4);
      const int off = tid < XU ? 32 * tid : 0x7fffffe0;
      xs[0][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
      xs[0][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, off + 16, 0, 0));
    } else {
      const auto rd = make_rsrc(dz3 + (size_t)b * 1568, 1568 * 4);
      const bool on = tid < DU && (tid >> 5) < 7;
      const int o = ((tid >> 5) * 7 * 32 + (tid & 31)) * 4;
#pragma unroll
      for (int e = 0; e < 7; ++e)
        ds[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rd, on ? o + 128 * e : 0x7ffffff0, 0, 0));
    }
  };
  auto fetch = [&](int b) {
    fetch_part(b, 0);
    fetch_part(b, 1);
  };
  auto put = [&](int buf, bool count) {   // count: add the dz to the bias partial
#pragma unroll
    for (int j = 0; j < XPER; ++j) {
      const int u = tid + NT * j;
      if (u < XU) {
        const int px = u >> 3, c = u & 7, y = px / 9, P = 12 * y + (px - 9 * y);
        const int off = P * 64 + 8 * (c ^ (2 * ((P >> 1) & 3)));
        Frag3 f;
        split8(xs[j][0], xs[j][1], f, false);
        *reinterpret_cast<bf16x8*>(&X[buf][off]) = f.h;
        *reinterpret_cast<bf16x8*>(&X[buf][XPL + off]) = f.m;
        *reinterpret_cast<bf16x8*>(&X[buf][2 * XPL + off]) = f.l;
      }
    }
    if (tid < DU) {
      Frag3 f;
      split8(f32x4{ds[0], ds[1], ds[2], ds[3]}, f32x4{ds[4], ds[5], ds[6], 0.f}, f, false);
#pragma unroll
      for (int e = 0; e < 7; ++e) bsum += count ? ds[e] : 0.f;
      const int off = (tid & 31) * DR + 8 * (tid >> 5);
      *reinterpret_cast<bf16x8*>(&D[buf][off]) = f.h;
      *reinterpret_cast<bf16x8*>(&D[buf][DPL + off]) = f.m;
      *reinterpret_cast<bf16x8*>(&D[buf][2 * DPL + off]) = f.l;
    }
  };
  f32x4 acc[3][2];   // [n tile][co tile]
#pragma unroll
  for (int j = 0; j < 3; ++j) acc[j][0] = acc[j][1] = zero4();
  const int Z = gridDim.x;
  int b = blockIdx.x, cur = 0;
  if (b < B) {
    fetch(b);
    put(0, true);
    fetch(b + Z < B ? b + Z : b);
  }
  __syncthreads();
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  for (; b < B; b += Z) {
    // every load in flight is this stage's (no stores in the loop): one explicit
    // wait, then the stage write unconditionally (past the end: not counted)
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
    put(cur ^ 1, b + Z < B);
    const int bnn = b + 2 * Z < B ? b + 2 * Z : b;
    const uint16_t* Xc = X[cur];
    const uint16_t* Dc = D[cur];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      Frag3 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int off = (16 * mt + i16) * DR + 32 * s + 8 * g;
        a[mt].h = *reinterpret_cast<const bf16x8*>(&Dc[off]);
        a[mt].m = *reinterpret_cast<const bf16x8*>(&Dc[DPL + off]);
        a[mt].l = *reinterpret_cast<const bf16x8*>(&Dc[2 * DPL + off]);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int n = 3 * wave + j, tap = n >> 2, ky = tap / 3, kx = tap - 3 * ky, cb = n & 3;
        s16x4 t[3][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int P = Pb[s][h] + 12 * ky + kx, unit = (4 * cb + p) ^ (4 * ((P >> 1) & 3));
          const uint16_t* rp = &Xc[P * 64 + 4 * unit];
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
  _Pragma("unroll") for (int mt = 0; mt < 2; ++mt) acc[j][mt] = mma(a[mt].XX, bf.YY, acc[j][mt]);
        PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
        if (s == 0 && j < 2) {
          fetch_part(bnn, j);
          __builtin_amdgcn_sched_barrier(0);   // the loads stay in their slot
        }
      }
    }
    __syncthreads();   // stage cur consumed; stage cur ^ 1 complete
    cur ^= 1;
  }
  // this block's partial: C row 4g + r of co tile mt, column i16 of n tile 3w + j
  float* o = slab + (size_t)blockIdx.x * (32 * 576) + 48 * wave + i16;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(16 * mt + 4 * g + r) * 576 + 16 * j] = acc[j][mt][r];
  if (tid < DU) bred[tid] = bsum;
  __syncthreads();
  if (tid < 32) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) t += bred[tid + 32 * w];
    slab_bias[(size_t)blockIdx.x * 32 + tid] = t;
  }
}

// conv2 dgrad, image-resident on the bf16 matrix cores (exact split, DESIGN.md
// §3): the phase-merged GEMM of Conv2Dgrad (n = (phase, ci), k = (tap, co)),
// one persistent block (8 waves) per CU walking images.  Per image the LDS holds
// dz2 already split into three bf16 planes, as a zero-padded 12 x 10 pixel grid
// (dz2 pixel (oy, ox) at (oy + 1, ox + 1); column 10 of a row is column 0 of the
// next, also zero): 2 stages x 51,840 B, the next image in flight into registers,
// so the k loop has no staging, no barrier and no range tests.  GEMM row m =
// 10 yy + xx is the dz1 phase pixel (yy, xx); its tap (ty, tx) is grid pixel
// m + 11 - (10 ty + tx).  A pixel is 144 B (64 co + 8 pad): 16 consecutive
// pixels start on 16 distinct 16-B bank slots (36 p mod 64, 9 odd), so the
// fragment reads are conflict-free without a swizzle and every (tile, k-step)
// offset is an immediate.
//   Border taps skipped: the rows run in 7 tiles — top row yy = 0 (10 pixels),
// five interior tiles (m = 10 .. 89, exact), bottom row yy = 9.  k-step s takes
// tap row ty = s & 1, lane group g = (tx = g & 1, co 16 (s >> 1) + 8 (g >> 1)):
// the top tile (ty = 1 reads only zero padding there) runs the even k-steps, the
// bottom tile (ty = 0) the odd ones: 48 tile-k-steps per image instead of 56 —
// 6 tiles every k-step (7 -> 1.87 ms per 65,536-image minibatch from 2.03).
// The k loop is software-pipelined over half k-steps (two groups of 3 tiles:
// the next group's fragments are read while the current group's MFMAs run;
// compute alone 1.41 -> 1.36 ms).  W2d [128][(ty, tx, co)] as packed: lane (n, g) of
// k-step s reads W2d[n][128 ty + 64 tx + 16 (s >> 1) + 8 (g >> 1) .. +7].
// Wave w owns n tile w (phase w >> 1, ci 16 (w & 1) + [0, 16)) for all of K,
// its weight fragments (pre-split planes, 8 k-steps x 3) in 96 VGPRs.
// Swapped operands (weights as A, pixels as B): lane (i16, g) holds row
// mrow(t) + i16 and the 4 consecutive channels 4g .. 4g+3 of its n tile — one
// 16-B store per tile; dummy rows get an out-of-range buffer offset (the store
// is dropped) instead of a branch.  The stores of image b are issued during
// image b + G's k-steps (one row tile per k-step) from registers masked at the
// end of image b, instead of all waves storing 51.2 KB at once before the barrier.
// BITS: the ReLU mask comes as bits (a1 points at u32 words [B][400] from
// ppo_conv1_fwd_mask, 1.6 KB per image) instead of the fp32 activations
// (51.2 KB per image): 40 % less HBM traffic, 12 % less time.
template <int NP, bool BITS = false, bool ANAT = false>
__global__ __launch_bounds__(512) void conv2_dgrad_x9_kernel(const float* __restrict__ dz2, int B,
                                                            const uint16_t* __restrict__ wpl,
                                                            const float* __restrict__ a1,
                                                            float* __restrict__ dz1, int stagger) {
  constexpr int HO = 9, CO = 64, GW = 10, GP = 12 * GW, PS = 72, PL = GP * PS, MT = 7, KS = 8;
  constexpr int CH = HO * HO * CO / 8, PER = (CH + 511) / 512, WN = 128 * 256;
  __shared__ __attribute__((aligned(16))) uint16_t S[2][3][PL];
  __shared__ int etab[16 * MT];   // row (t, i16) -> output offset yy*1280 + xx*64 (or -1: dummy row)
  // ReLU mask of a1 (conv1's output) for the image: bits, or one byte per
  // element, staged like dz2 (coalesced 16-B loads one image ahead, in registers)
  constexpr int MC = BITS ? 400 : 400 * 32 / 4, MPER = (MC + 511) / 512;
  __shared__ __attribute__((aligned(16))) uint32_t Mk[2][MC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, i16 = lane & 15, g = lane >> 4;
  const int n = 16 * wave + i16, ph = wave >> 1;
  constexpr auto mrow = [](int t) { return t == 0 ? 0 : t == MT - 1 ? 90 : 16 * t - 6; };
  bf16x8 bw[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      bw[s][p] = *reinterpret_cast<const bf16x8*>(wpl + (size_t)p * WN + n * 256 + 128 * (s & 1) + 64 * (g & 1) +
                                                  16 * (s >> 1) + 8 * (g >> 1));
  wait_vm0();
  // zero the pad pixels of both stages (staging only ever writes the 81 real ones)
  for (int i = tid; i < 2 * 3 * GP * 9; i += 512) {
    const int c = i % (GP * 9), p = c / 9, py = p / GW, px = p - GW * py;
    if (py == 0 || py >= 10 || px == 0)
      *reinterpret_cast<uint4*>(&S[i / (3 * GP * 9)][(i / (GP * 9)) % 3][8 * c]) = uint4{0, 0, 0, 0};
  }
  if (tid < 16 * MT) {
    const int t = tid >> 4, r = tid & 15, m = mrow(t) + r;
    etab[tid] = ((t == 0 || t == MT - 1) && r >= 10) ? -1 : (m / 10) * 1280 + (m % 10) * 64;
  }
  // byte offset of this lane's fragment at row 0, ty 0, k-step 0; (tile t, k-step
  // s) adds 144 (mrow(t) - 10 (s & 1)) + 32 (s >> 1): an immediate
  const int abase = (i16 + 11 - (g & 1)) * (2 * PS) + 16 * (g >> 1);
  f32x4 stg[PER][2];
  f32x4 mst[BITS ? 1 : MPER];
  uint4 mbv;
  // part j of an image's loads: dz2 unit j (+ the mask bits with the last one)
  auto fetch_part = [&](int b, int j) {
    const f32x4* src = reinterpret_cast<const f32x4*>(dz2 + (size_t)b * (HO * HO * CO));
    const int c = tid + 512 * j;
    const int cc = c < CH ? c : 0;   // unconditional loads: no exec branch around them
    stg[j][0] = src[2 * cc];
    stg[j][1] = src[2 * cc + 1];
    if constexpr (BITS) {
      if (j == PER - 1) {   // 400 words; lanes past them read out of range (0), no branch
        const auto rm = make_rsrc(reinterpret_cast<const uint32_t*>(a1) + (size_t)b * 400, 1600);
        mbv = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rm, tid < 100 ? 16 * tid : 0x7ffffff0,
                                                                              0, 0));
      }
    }
  };
  auto fetch = [&](int b) {
    if constexpr (BITS) {
#pragma unroll
      for (int j = 0; j < PER; ++j) fetch_part(b, j);
    } else {
      const f32x4* src = reinterpret_cast<const f32x4*>(dz2 + (size_t)b * (HO * HO * CO));
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int c = tid + 512 * j;
        const int cc = c < CH ? c : 0;
        stg[j][0] = src[2 * cc];
        stg[j][1] = src[2 * cc + 1];
      }
      const f32x4* ms = reinterpret_cast<const f32x4*>(a1 + (size_t)b * 12800);
#pragma unroll
      for (int j = 0; j < MPER; ++j) {
        const int c = tid + 512 * j;
        if (c < MC) mst[j] = ms[c];
      }
    }
  };
  auto put = [&](int buf) {
    if constexpr (BITS) {
      if (tid < 100) reinterpret_cast<uint4*>(Mk[buf])[tid] = mbv;
    } else {
#pragma unroll
      for (int j = 0; j < MPER; ++j) {
        const int c = tid + 512 * j;
        if (c < MC)
          Mk[buf][c] = (mst[j][0] > 0.f ? 1u : 0u) | (mst[j][1] > 0.f ? 0x100u : 0u) |
                       (mst[j][2] > 0.f ? 0x10000u : 0u) | (mst[j][3] > 0.f ? 0x1000000u : 0u);
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int c = tid + 512 * j;
      if (c < CH) {
        const int r = c >> 3, oy = r / HO, p = (oy + 1) * GW + (r - HO * oy) + 1;
        const int off = p * PS + 8 * (c & 7);
        Frag3 f;
        split8(stg[j][0], stg[j][1], f, false);
        *reinterpret_cast<bf16x8*>(&S[buf][0][off]) = f.h;
        *reinterpret_cast<bf16x8*>(&S[buf][1][off]) = f.m;
        *reinterpret_cast<bf16x8*>(&S[buf][2][off]) = f.l;
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
  const bool late = (stagger & 1) && wave >= 4;   // waves 4-7 stage after their compute (see conv3 dgrad; !BITS)
  // timing anatomy only (tools/kbench.py --tune stagger=...; wrong results):
  // 16 skips the MFMAs, 32 the epilogue stores, 64 the staging of the next image (!BITS)
  // (compiled in only for ANAT: a runtime branch around the k loop costs the
  // default kernel exact wait counts at its merge)
  const bool no_mma = ANAT && (stagger & 16), no_epi = ANAT && (stagger & 32), no_stage = ANAT && (stagger & 64);
  f32x4 eacc[MT];
  int bprev = -1;
  const int cbs = (ph >> 1) * 640 + (ph & 1) * 32 + 16 * (wave & 1) + 4 * g;
  // (bp < 0: before the first image, or no_epi: an empty range drops the store)
  auto store_tile = [&](int t, const f32x4& v, int bp) {
    const int eo = etab[16 * t + i16];
    const auto rs = make_rsrc(dz1 + (size_t)max(bp, 0) * 12800, bp >= 0 && !no_epi ? 12800 * 4 : 0);
    bstore_f32x4(v, rs, eo >= 0 ? 4 * (eo + cbs) : -1);
  };
  for (; b < B; b += G) {
    // BITS: branch-free staging (a conditional load made the wait counts unknown
    // at the merge): the next image's stage is written unconditionally and the
    // image after next (the block's last image re-read past the end) is loaded in
    // two parts during k-steps 1 and 3, not all at once before the k loop
    const int bnn = b + 2 * G < B ? b + 2 * G : b;
    if constexpr (BITS) {
      // every load in flight is this stage's (issued a k-step or more ago): wait
      // for all of them here, or the partial unit's exec branch in put leaves them
      // pending on one path and the fragment reads below wait one by one
      __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0) (expcnt / lgkmcnt unconstrained)
      put(cur ^ 1);
    } else if (!late && !no_stage) {
      if (b + G < B) put(cur ^ 1);
      if (b + 2 * G < B) fetch(b + 2 * G);
    }
    const char* Sb = reinterpret_cast<const char*>(S[cur][0]) + abase;
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = zero4();
    if (no_mma) {   // anatomy only
#pragma unroll
      for (int t = 0; t < MT; ++t) store_tile(t, eacc[t], bprev);
      if constexpr (BITS) fetch(bnn);
    } else {
      // software pipeline over half k-steps: group 0 = {border tile of the tap
      // row, tiles 1, 2}, group 1 = tiles 3-5; the fragments of the next group
      // are read while the current one's MFMAs run (2 x 36 VGPRs)
      Frag3 fr[2][3];
      auto tile_of = [](int s, int grp, int u) {
        return grp == 0 ? (u == 0 ? ((s & 1) ? MT - 1 : 0) : u) : 3 + u;
      };
      auto ld = [&](int s, int grp) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int t = tile_of(s, grp, u);
          const char* q = Sb + 2 * PS * (mrow(t) - 10 * (s & 1)) + 32 * (s >> 1);
          fr[grp][u].h = *reinterpret_cast<const bf16x8*>(q);
          fr[grp][u].m = *reinterpret_cast<const bf16x8*>(q + 2 * PL);
          fr[grp][u].l = *reinterpret_cast<const bf16x8*>(q + 4 * PL);
        }
      };
      auto mm = [&](int s, int grp) {
        const Frag3 w = {bw[s][0], bw[s][1], bw[s][2]};
#define PPO_PART(X, Y)                                                                \
  _Pragma("unroll") for (int u = 0; u < 3; ++u) {                                     \
    const int t = tile_of(s, grp, u);                                                 \
    acc[t] = mma(w.Y, fr[grp][u].X, acc[t]);                                          \
  }
        PPO_PRODUCTS(NP, PPO_PART)
#undef PPO_PART
      };
      // (the fp32-mask variant holds 28 more VGPRs of mask staging: no pipeline)
      if constexpr (BITS) ld(0, 0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if constexpr (BITS) {
          ld(s, 1);
          __builtin_amdgcn_sched_barrier(0);
          mm(s, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (s + 1 < KS) ld(s + 1, 0);
          __builtin_amdgcn_sched_barrier(0);
          mm(s, 1);
        } else {
          ld(s, 0);
          mm(s, 0);
          ld(s, 1);
          mm(s, 1);
        }
        if constexpr (BITS) {
          if (s < MT) store_tile(s, eacc[s], bprev);
          if (s == 1 || s == 3) fetch_part(bnn, s >> 1);
          __builtin_amdgcn_sched_barrier(0);
        } else if (s < MT && bprev >= 0 && !no_epi) {
          store_tile(s, eacc[s], bprev);
        }
      }
    }
    // masked results of this image, stored during the next one's k-steps:
    // C row 4g + r of the swapped tile is channel 4g + r of pixel row (t, i16)
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int i = max(etab[16 * t + i16], 0) + cbs;   // element (pixel i >> 5, channels (i & 31) + r)
      const uint32_t mw = Mk[cur][i >> 5] >> (i & 31);
      const uint8_t* mk = reinterpret_cast<const uint8_t*>(Mk[cur]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool keep = BITS ? ((mw >> r) & 1u) != 0 : mk[i + r] != 0;
        eacc[t][r] = keep ? acc[t][r] : 0.f;
      }
    }
    bprev = b;
    if (!BITS && late && !no_stage) {
      if (b + G < B) put(cur ^ 1);
      if (b + 2 * G < B) fetch(b + 2 * G);
    }
    __syncthreads();   // every wave is done with S[cur]; S[cur ^ 1] is complete
    cur ^= 1;
  }
  if (bprev >= 0 && !no_epi) {
#pragma unroll
    for (int t = 0; t < MT; ++t) store_tile(t, eacc[t], bprev);
  }
}

// ---------------------------------------------------------------------------
// Weight-gradient (wgrad) problems: dW[co][kk] = Σ_r dz[r][co] · X(r, kk)
// over the reduction r = (b, output pixel), split over blockIdx.z into fp32
// partial slabs (deterministic sum in ppo_wgrad_reduce).  Both operands are
// row-contiguous tiles; blocks of tile column 0 also sum the dz tile into the
// bias partial (db[co] = Σ_r dz[r][co]).
// ---------------------------------------------------------------------------
// conv1 wgrad: X(r, kk) = decoded obs[idx[b]][c][4oy+ky][4ox+kx], kk = (c,ky,kx)
// A k-tile (BK rows, BK | 400, chunks BK-aligned) never straddles two images,
// so the image (and its minibatch row gather) is resolved once per tile from
// the block-uniform tile start — a scalar load, not one per operand load.
template <typename InT, class C_>
struct Conv1Wgrad : WgradBase<C_> {
  static_assert(400 % C_::BK == 0, "conv1 wgrad k-tiles must not straddle images");
  static constexpr bool B_TILE = true;
  const InT* obs; const int64_t* idx; long long row0; int C;
  struct BCtx { int off; bool ok; };
  struct TCtx { const InT* img; int r0; };
  using Raw = std::conditional_t<sizeof(InT) == 1, uint32_t, f32x4>;
  __device__ BCtx b_ctx(int n, int) const {
    const int ch = n >> 6, ky = (n >> 3) & 7, kx = n & 7;
    return {ch * IMG2 + ky * IMG + kx, n < C * 64};
  }
  __device__ TCtx tile(int k0) const {
    const int b = k0 / 400;
    return {obs + obs_row(idx, row0, b) * (long long)(C * IMG2), b * 400};
  }
  __device__ Raw b_load_t(const BCtx& c, const TCtx& t, int r) const {
    if (!c.ok || r >= this->R) return Raw{};
    const int pp = r - t.r0, oy = pp / 20, ox = pp - oy * 20;
    return *reinterpret_cast<const Raw*>(t.img + (oy * 4) * IMG + ox * 4 + c.off);
  }
};

// Pack torch-layout weights into the loaders' k orders (once per optimizer step).
//   W2p [64][512]  (ky,kx,ci)       W3p [32][576] (ky,kx,ci)
//   W4p [H][1568]  (p,c)            W4T [1568][H] (p,c) x n
//   W3d [64][288]  ci x (ky,kx,co)  W2d [4][32][256] phase x ci x (ty,tx,co)
// Each f32 segment of n values is followed by its exact bf16 split (hi, mid, lo
// planes of n bf16 each = 1.5 n floats), the B operand of the igemm_x9 core.
__host__ __device__ inline void pack_segments(int H, long long* n) {
  n[0] = 64 * 512; n[1] = 32 * 576; n[2] = (long long)H * 1568; n[3] = n[2]; n[4] = 64 * 288; n[5] = 4 * 32 * 256;
}

__global__ __launch_bounds__(256) void pack_weights_kernel(const float* __restrict__ w2, const float* __restrict__ w3,
                                                           const float* __restrict__ w4, int H,
                                                           float* __restrict__ out) {
  long long n[6];
  pack_segments(H, n);
  const long long total = n[0] + n[1] + n[2] + n[3] + n[4] + n[5];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    long long j = i, base = 0;
    int seg = 0;
    while (j >= n[seg]) {
      j -= n[seg];
      base += n[seg] * 5 / 2;
      ++seg;
    }
    float v;
    if (seg == 0) {
      const int co = (int)(j / 512), k = (int)(j % 512), ky = k / 128, kx = (k / 32) % 4, ci = k % 32;
      v = w2[co * 512 + ci * 16 + ky * 4 + kx];
    } else if (seg == 1) {
      const int co = (int)(j / 576), k = (int)(j % 576), ky = k / 192, kx = (k / 64) % 3, ci = k % 64;
      v = w3[co * 576 + ci * 9 + ky * 3 + kx];
    } else if (seg == 2) {
      const long long nn = j / 1568;
      const int k = (int)(j % 1568), pp = k / 32, c = k % 32;
      v = w4[nn * 1568 + c * 49 + pp];
    } else if (seg == 3) {
      const int k = (int)(j / H), nn = (int)(j % H), pp = k / 32, c = k % 32;
      v = w4[(long long)nn * 1568 + c * 49 + pp];
    } else if (seg == 4) {
      const int ci = (int)(j / 288), k = (int)(j % 288), ky = k / 96, kx = (k / 32) % 3, co = k % 32;
      v = w3[co * 576 + ci * 9 + ky * 3 + kx];
    } else {
      const int ph = (int)(j / 8192), rem = (int)(j % 8192), ci = rem / 256, k = rem % 256;
      const int ty = k >> 7, tx = (k >> 6) & 1, co = k & 63;
      const int ky = (ph >> 1) + 2 * ty, kx = (ph & 1) + 2 * tx;
      v = w2[co * 512 + ci * 16 + ky * 4 + kx];
    }
    out[base + j] = v;
    uint32_t h, m, l;
    split_bf16x3(v, h, m, l);
    uint16_t* pl = reinterpret_cast<uint16_t*>(out + base + n[seg]);
    pl[j] = (uint16_t)h;
    pl[n[seg] + j] = (uint16_t)m;
    pl[2 * n[seg] + j] = (uint16_t)l;
  }
}

using CfgN64 = Cfg<128, 64, 2, 2, true, true>;
using CfgN128 = Cfg<128, 128, 2, 2, true, true>;

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
// floats: every segment is followed by its three bf16 planes (1.5 x its size)
PPO_API long long ppo_packed_weights_size(int H) {
  long long n[6];
  pack_segments(H, n);
  return (n[0] + n[1] + n[2] + n[3] + n[4] + n[5]) * 5 / 2;
}

// offsets (floats) of the packed f32 segments W2p W3p W4p W4T W3d W2d inside the pack buffer
PPO_API int ppo_packed_offsets(int H, long long* off6) {
  long long n[6];
  pack_segments(H, n);
  off6[0] = 0;
  for (int i = 1; i < 6; ++i) off6[i] = off6[i - 1] + n[i - 1] * 5 / 2;
  return 0;
}

// bf16 planes of a packed segment of n floats (they follow it)
static inline const uint16_t* planes_of(const float* seg, long long n) {
  return reinterpret_cast<const uint16_t*>(seg + n);
}

PPO_API int ppo_pack_weights(const float* w2, const float* w3, const float* w4, int H, float* packed, void* stream) {
  ProfScope prof("pack_weights", as_stream(stream), 4.0 * 4.0 * ppo_packed_weights_size(H));
  PPO_REQUIRE(H > 0 && H % 4 == 0, "ppo_pack_weights: hidden size %d must be a positive multiple of 4", H);
  long long n[6];
  pack_segments(H, n);
  const long long total = n[0] + n[1] + n[2] + n[3] + n[4] + n[5];
  long long b = (total + 255) / 256;
  pack_weights_kernel<<<(unsigned)(b < 2048 ? b : 2048), 256, 0, as_stream(stream)>>>(w2, w3, w4, H, packed);
  PPO_LAUNCH_CHECK("pack_weights_kernel");
  return 0;
}

// ---------------------------------------------------------------------------
// Run-time knobs (ppo_tune_set / ppo_tune_get).  Each selects between the default
// kernel and one kept alternative that a test or a documented A/B depends on;
// the superseded variants of rounds 1-4 live in git history, not in the library.
//   conv1_fwd    0: image-resident bf16x3 kernel (u8, C = 4); 9: the generic tile GEMM
//                (the path any other C takes), for A/B and its parity test
//   conv1_wgrad  9: k-split kernel with one wave per SIMD (conv1w.hip, default since
//                round 5); 10: its two-waves-per-SIMD form; 8: the round-4 k-split
//                kernel (8 waves, u8 image by LDS-DMA); 5: part-pipelined kernel (the
//                half-precision mode's, bf16 dz)
//   x9           1: fp32 GEMMs on the bf16 matrix cores (exact split, igemm_x9.h) where
//                they measured faster; 0: fp32 MFMA (igemm.h); 2: the split core everywhere
//   fc_splitk    K slices of the rollout-sized fc forward with a workspace (<= 1: unsplit)
//   rgb_aff      1: conv1 on raw RGB frames by the affine fold (rgbaff.hip); 0: bit-exact decode
//   fc_splitk_tile 1: the rollout's split-K fc on 128 x 128 tiles (4 waves of 32 x 128), 16-B
//                slab stores; 0: 128 x 64 tiles (8 waves of 16 x 64), 4-B stores
// ---------------------------------------------------------------------------
enum { TK_CONV1_FWD, TK_CONV1_WGRAD, TK_X9, TK_FC_SPLITK, TK_RGB_AFF, TK_FC_SPLITK_TILE, TK_N };
static const char* g_tune_names[TK_N] = {"conv1_fwd", "conv1_wgrad", "x9", "fc_splitk", "rgb_aff", "fc_splitk_tile"};
// fc_splitk 4 with 128 x 128 tiles: 0.050-0.052 vs 0.054-0.055 ms per 4,096-row act for 2
// slices of 128 x 64 tiles (profiles/r06_s7_fc_splitk_sweep.log)
static int g_tune[TK_N] = {0, 9, 1, 4, 1, 1};
// stagger: the image-resident kernels with two LDS stages let waves 4-7 stage the
// next image after their compute (conv2 / conv3 dgrad, conv3 forward)
static int g_stagger = 2;   // bit 1 (conv2 dgrad deferred 16-B stores): measured best
// small_b: forwards of at most this many samples (images / linear rows) take the
// small-batch path of small.hip (an output element per thread or wave, fp32 FMA)
static int g_small_b = 4;

static bool tune_ok(int k, int v) {
  switch (k) {
    case TK_CONV1_FWD: return v == 0 || v == 9;
    case TK_CONV1_WGRAD: return v == 5 || v == 8 || v == 9 || v == 10;
    case TK_X9: return v >= 0 && v <= 2;
    case TK_FC_SPLITK: return v >= 0 && v <= 8;
    case TK_FC_SPLITK_TILE: return v == 0 || v == 1;
    default: return v == 0 || v == 1;
  }
}

int heads_lds_knob(int set, int value);   // heads.hip (the LDS-weight heads_train kernel, default on)

PPO_API int ppo_tune_set(const char* key, int value) {
  if (strcmp(key, "heads_lds") == 0) {
    heads_lds_knob(1, value);
    return 0;
  }
  if (strcmp(key, "small_b") == 0) {
    PPO_REQUIRE(value >= 0, "ppo_tune_set: small_b must be >= 0, got %d", value);
    g_small_b = value;
    return 0;
  }

  if (strcmp(key, "stagger") == 0) {
#ifndef PPO_DIAG
    // bits 0-3 are schedule switches (same results); bits >= 4 select the timing-
    // anatomy paths of diagnostic kernels (wrong results by design): -DPPO_DIAG only
    PPO_REQUIRE(value >= 0 && value < 16, "ppo_tune_set: stagger takes schedule bits 0..15, got %d "
                "(the anatomy bits need a -DPPO_DIAG build)", value);
#endif
    g_stagger = value;
    return 0;
  }
  if (strcmp(key, "products") == 0) {
    PPO_REQUIRE(value == 1 || value == 6 || value == 9, "ppo_tune_set: products must be 1, 6 or 9, got %d", value);
    g_products = value;
    return 0;
  }
  for (int i = 0; i < TK_N; ++i)
    if (strcmp(key, g_tune_names[i]) == 0) {
      PPO_REQUIRE(tune_ok(i, value), "ppo_tune_set: %s = %d is not a kept variant", key, value);
      g_tune[i] = value;
      return 0;
    }
  ppo_set_error("ppo_tune_set: unknown key %s", key);
  return PPO_EARG;
}

PPO_API int ppo_tune_get(const char* key) {
  if (strcmp(key, "heads_lds") == 0) return heads_lds_knob(0, 0);
  if (strcmp(key, "small_b") == 0) return g_small_b;
  if (strcmp(key, "stagger") == 0) return g_stagger;
  if (strcmp(key, "products") == 0) return g_products;
  for (int i = 0; i < TK_N; ++i)
    if (strcmp(key, g_tune_names[i]) == 0) return g_tune[i];
  return -1;
}

// fp32-MFMA tile core (x9 = 0 and the generic fallbacks): the measured best tile
// of the round-1 sweep (profiles/r01_kbench_sweep_v2.log) for the N = 32 problem
using V32_0 = Cfg<256, 32, 4, 1, true, true>;           // 4 waves x 64 rows, 46 KB LDS

// exact-split bf16 core (igemm_x9.h)
using X64 = CfgX<128, 64, 2, 2, true, true>;          // N = 64: waves of 64x32
using X128 = CfgX<128, 128, 2, 2, true, true>;        // N >= 128: waves of 64x64
using X64s = CfgX<64, 64, 2, 2, true, true>;          // few 128 x 128 tiles (rollout rows): waves of 32x32
using XW64 = CfgX<64, 128, 2, 2, false, false, true>;   // wgrad, 64 output channels
using XP128 = CfgX<128, 128, 4, 1, true, true, false, false, false, true>;  // B from planes, waves 32x128
using XP128w8 = CfgX<128, 128, 8, 1, true, true, false, false, false, true>;      // 8 waves of 16x128
using XP128x64w8 = CfgX<128, 64, 8, 1, true, true, false, false, false, true>;    // 8 waves of 16x64 (2 blocks/CU)
// split-at-staging form (igemm_x9s_kernel): both operands split once per block into bf16 planes in LDS
using SW256x128 = CfgS<256, 128, 4, 2, false, false, true>;      // wgrad: 8 waves of 64x64 (144 KB LDS)

// compute units of the current device (persistent-kernel grid size)
static int device_cus() {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    n_cu = n;
  }
  return n_cu;
}

// x9 = 1: the split-bf16 core where it measured faster (the dense forward / dgrad, the
// fc weight gradient); x9 = 2: also the narrow GRU / MLP weight gradients; 0: fp32 MFMA
static inline bool use_x9() { return g_tune[TK_X9] != 0; }
static inline bool use_x9_all() { return g_tune[TK_X9] == 2; }
template <class P>
static inline void set_planes(P& p, const float* seg, long long n, int rows, int K) {
  p.bpl = planes_of(seg, n); p.bps = n; p.bld = K; p.bnr = rows;
}

// persistent image-resident grid: one block per CU (fewer for a small batch)
static inline unsigned img_grid(int B) {
  const int n_cu = device_cus();
  return (unsigned)(B < n_cu ? B : n_cu);
}

static int conv1_fwd_impl(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                          const float* w1, const float* b1, float* out, uint16_t* mbits, void* stream);
int conv1_wgrad_kw(const float* dz1, const uint8_t* obs, const int64_t* idx, long long row0, int B, int Z,
                   float* slab, float* slab_bias, void* stream);
int conv1_wgrad_kw3(const float* dz1, const uint8_t* obs, const int64_t* idx, long long row0, int B, int Z,
                   float* slab, float* slab_bias, void* stream, int nw);   // conv1w.hip

// conv1 forward: out [B][20][20][32] = relu(conv(obs rows, W1 torch layout) + b1)
PPO_API int ppo_conv1_fwd(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                          const float* w1, const float* b1, float* out, void* stream) {
  return conv1_fwd_impl(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, nullptr, stream);
}

// conv1 forward that also writes the ReLU mask of its output as bits
// (mbits [B][400] u32, bit c of pixel p = out[p][c] > 0) for ppo_conv2_dgrad_bits.
PPO_API int ppo_conv1_fwd_mask(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                               const float* w1, const float* b1, float* out, uint32_t* mbits, void* stream) {
  PPO_REQUIRE(mbits != nullptr, "ppo_conv1_fwd_mask: null mask");
  return conv1_fwd_impl(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, reinterpret_cast<uint16_t*>(mbits), stream);
}

static int conv1_fwd_impl(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                          const float* w1, const float* b1, float* out, uint16_t* mbits, void* stream) {
  PPO_REQUIRE(B >= 0 && C > 0, "ppo_conv1_fwd: B=%d C=%d", B, C);
  if (!mbits && B > 0 && B <= g_small_b)
    return small_conv1_fwd(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, as_stream(stream));
  // float observations (the reference's fp32 storage plane): the image-resident
  // split-bf16 kernel of conv1f.hip
  if (!obs_is_u8 && C == 4 && ((uintptr_t)obs & 15) == 0)
    return ppo_conv1_fwd_f32((const float*)obs, idx, row0, B, w1, b1, out, reinterpret_cast<uint32_t*>(mbits), stream);
  const bool img = obs_is_u8 && C == 4 && g_tune[TK_CONV1_FWD] == 0;
  if (mbits && !img) {
    // the generic path has no fused mask epilogue: the conv, then the mask from its output
    const int rc = conv1_fwd_impl(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, nullptr, stream);
    if (rc != 0 || B == 0) return rc;
    const long long halves = (long long)B * 800;
    const long long nb = (halves + 255) / 256;
    relu_bits_kernel<<<(unsigned)(nb < 8192 ? nb : 8192), 256, 0, as_stream(stream)>>>(out, halves, mbits);
    PPO_LAUNCH_CHECK("relu_bits_kernel");
    return 0;
  }
  const long long M = (long long)B * 400;
  const double fl = 2.0 * M * 32 * C * 64;
  if (img) {
    if (B == 0) return 0;
    const unsigned nb = img_grid(B);
    int slot;
    const bool prof = ppo_prof_begin("conv1_fwd_u8", as_stream(stream), &slot);
    const uint8_t* o8 = (const uint8_t*)obs;
    hipStream_t st = as_stream(stream);
    if (g_products == 1) {   // half-precision mode: bf16 weights
      if (mbits) conv1_fwd_bf16x3_kernel<4, true, 1><<<nb, 512, 0, st>>>(o8, idx, row0, B, w1, b1, out, mbits);
      else conv1_fwd_bf16x3_kernel<4, false, 1><<<nb, 512, 0, st>>>(o8, idx, row0, B, w1, b1, out, nullptr);
    } else if (mbits) {
      conv1_fwd_bf16x3_kernel<4, true><<<nb, 512, 0, st>>>(o8, idx, row0, B, w1, b1, out, mbits);
    } else {
      conv1_fwd_bf16x3_kernel<4, false><<<nb, 512, 0, st>>>(o8, idx, row0, B, w1, b1, out, nullptr);
    }
    if (prof) ppo_prof_end(slot, st, fl);
    PPO_LAUNCH_CHECK("conv1_fwd_u8 (image-resident)");
    return 0;
  }
#define SETUP1(T_)                                                                                 \
  p.obs = (const T_*)obs; p.idx = idx; p.row0 = row0; p.C = C; p.M = (int)M; p.w = w1; p.bias = b1; p.out = out
  if (obs_is_u8) {
    Conv1Fwd<uint8_t, V32_0> p;
    SETUP1(uint8_t);
    return launch(p, M, 32, 1, as_stream(stream), "conv1_fwd_u8", fl);
  }
  Conv1Fwd<float, V32_0> p;
  SETUP1(float);
  return launch(p, M, 32, 1, as_stream(stream), "conv1_fwd_f32", fl);
#undef SETUP1
}

static int conv2_fwd_impl(const float* a1, int B, const float* w2p, const float* b2, float* out, uint16_t* mbits,
                          void* stream) {
  if (!mbits && B > 0 && B <= g_small_b) return small_conv2_fwd(a1, B, w2p, b2, out, as_stream(stream));
  if (B <= 0) return 0;
  const unsigned nb = img_grid(B);
  int slot;
  const bool prof = ppo_prof_begin("conv2_fwd", as_stream(stream), &slot);
  const uint16_t* wpl = planes_of(w2p, 64 * 512);
  hipStream_t st = as_stream(stream);
  if (mbits && g_products == 9) conv2_fwd_x9c_kernel<9, true><<<nb, 512, 0, st>>>(a1, B, wpl, b2, out, mbits);
  else if (mbits && g_products == 1) conv2_fwd_x9c_kernel<1, true><<<nb, 512, 0, st>>>(a1, B, wpl, b2, out, mbits);
  else if (mbits) conv2_fwd_x9c_kernel<6, true><<<nb, 512, 0, st>>>(a1, B, wpl, b2, out, mbits);
  else PPO_LAUNCH_NP(conv2_fwd_x9c_kernel, nb, 512, st, a1, B, wpl, b2, out, nullptr);
  if (C2F_LONE == 1) {   // output pixel 72 of every image in a launch of its own
    const int ntile = (B + 15) / 16;
    const unsigned nl = (unsigned)(ntile < 512 ? ntile : 512);
    if (mbits && g_products == 9) conv2_fwd_lone_kernel<9, true><<<nl, 512, 0, st>>>(a1, B, wpl, b2, out, mbits);
    else if (mbits && g_products == 1) conv2_fwd_lone_kernel<1, true><<<nl, 512, 0, st>>>(a1, B, wpl, b2, out, mbits);
    else if (mbits) conv2_fwd_lone_kernel<6, true><<<nl, 512, 0, st>>>(a1, B, wpl, b2, out, mbits);
    else if (g_products == 9) conv2_fwd_lone_kernel<9, false><<<nl, 512, 0, st>>>(a1, B, wpl, b2, out, nullptr);
    else if (g_products == 1) conv2_fwd_lone_kernel<1, false><<<nl, 512, 0, st>>>(a1, B, wpl, b2, out, nullptr);
    else conv2_fwd_lone_kernel<6, false><<<nl, 512, 0, st>>>(a1, B, wpl, b2, out, nullptr);
  }
  if (prof) ppo_prof_end(slot, st, 2.0 * B * 81 * 64 * 512);
  PPO_LAUNCH_CHECK("conv2_fwd_x9c_kernel");
  return 0;
}

PPO_API int ppo_conv2_fwd(const float* a1, int B, const float* w2p, const float* b2, float* out, void* stream) {
  return conv2_fwd_impl(a1, B, w2p, b2, out, nullptr, stream);
}

// conv2 forward that also writes the ReLU mask of its output as bits
// (mbits [B][81] u64, bit c of pixel p = out[p][c] > 0) for ppo_conv3_dgrad_bits.
PPO_API int ppo_conv2_fwd_mask(const float* a1, int B, const float* w2p, const float* b2, float* out,
                               uint64_t* mbits, void* stream) {
  PPO_REQUIRE(mbits != nullptr, "ppo_conv2_fwd_mask: null mask");
  return conv2_fwd_impl(a1, B, w2p, b2, out, reinterpret_cast<uint16_t*>(mbits), stream);
}

static int conv3_fwd_impl(const float* a2, int B, const float* w3p, const float* b3, float* out, uint16_t* m3,
                          void* stream) {
  if (B > 0 && B <= g_small_b && !m3) return small_conv3_fwd(a2, B, w3p, b3, out, as_stream(stream));
  if (B <= 0) return 0;
  int slot;
  const bool prof = ppo_prof_begin("conv3_fwd", as_stream(stream), &slot);
  const uint16_t* wpl = planes_of(w3p, 32 * 576);
  if (C3F_COMPACT || m3) {   // compact rows (three tiles) + the lone output (6, 6)
    PPO_LAUNCH_NP(conv3_fwd_c3_kernel, img_grid(B), 768, as_stream(stream), a2, B, wpl, b3, out, m3);
    if (C3F_COMPACT == 1 && !m3) {
      const int ntile = (B + 15) / 16;
      PPO_LAUNCH_NP(conv3_fwd_lone_kernel, (unsigned)(ntile < 512 ? ntile : 512), 256, as_stream(stream), a2, B,
                    wpl, b3, out);
    }
  } else {
    PPO_LAUNCH_NP(conv3_fwd_x9_kernel, img_grid(B), 512, as_stream(stream), a2, B, wpl, b3, out, g_stagger);
  }
  if (prof) ppo_prof_end(slot, as_stream(stream), 2.0 * B * 49 * 32 * 576);
  PPO_LAUNCH_CHECK("conv3_fwd_x9_kernel");
  return 0;
}

PPO_API int ppo_conv3_fwd(const float* a2, int B, const float* w3p, const float* b3, float* out, void* stream) {
  return conv3_fwd_impl(a2, B, w3p, b3, out, nullptr, stream);
}

// the training forward: also the ReLU mask bits of the output, uint16 [B][49][2]
// (conv3_mask_store), read by ppo_fc_dgrad_bits
PPO_API int ppo_conv3_fwd_mask(const float* a2, int B, const float* w3p, const float* b3, float* out,
                               uint16_t* mbits, void* stream) {
  PPO_REQUIRE(mbits != nullptr, "ppo_conv3_fwd_mask: null mask");
  return conv3_fwd_impl(a2, B, w3p, b3, out, mbits, stream);
}

// conv1 -> conv2 -> conv3 forward (model.py:177-179) of u8 4-channel observation rows in
// one launch (trunk_fwd_kernel): a1, a2, a3 as ppo_conv1_fwd / ppo_conv2_fwd /
// ppo_conv3_fwd write them (bit-identical); m1 / m2 both NULL or both given (the
// ReLU mask bits of ppo_conv1_fwd_mask / ppo_conv2_fwd_mask).  Small batches (<=
// small_b) and conv1_fwd tune 9 take the three separate calls.
PPO_API int ppo_trunk_fwd(const uint8_t* obs, const int64_t* idx, long long row0, int B, const float* w1,
                          const float* b1, float* a1, uint32_t* m1, const float* w2p, const float* b2, float* a2,
                          uint64_t* m2, const float* w3p, const float* b3, float* a3, void* stream) {
  PPO_REQUIRE(B >= 0 && obs != nullptr && (m1 == nullptr) == (m2 == nullptr),
              "ppo_trunk_fwd: B=%d, obs and both-or-neither masks required", B);
  if (B == 0) return 0;
  // the masked (training) form runs the three launches: fused, its registers spill
  // (2 VGPRs at 256), and the training forward has 2 boundaries per minibatch only
  if (B <= g_small_b || g_tune[TK_CONV1_FWD] != 0 || m1 != nullptr) {
    int rc = conv1_fwd_impl(obs, 1, idx, row0, 4, B, w1, b1, a1, reinterpret_cast<uint16_t*>(m1), stream);
    if (rc == 0) rc = conv2_fwd_impl(a1, B, w2p, b2, a2, reinterpret_cast<uint16_t*>(m2), stream);
    if (rc == 0) rc = ppo_conv3_fwd(a2, B, w3p, b3, a3, stream);
    return rc;
  }
  const unsigned nb = img_grid(B);
  hipStream_t st = as_stream(stream);
  int slot;
  const bool prof = ppo_prof_begin("trunk_fwd", st, &slot);
  const uint16_t* w2pl = planes_of(w2p, 64 * 512);
  const uint16_t* w3pl = planes_of(w3p, 32 * 576);
#define PPO_TRUNK(NP_) \
  trunk_fwd_kernel<NP_, false><<<nb, 512, 0, st>>>(obs, idx, row0, B, w1, b1, a1, nullptr, w2pl, b2, a2, nullptr, \
                                                    w3pl, b3, a3)
  if (g_products == 9) PPO_TRUNK(9);
  else if (g_products == 1) PPO_TRUNK(1);
  else PPO_TRUNK(6);
#undef PPO_TRUNK
  if (prof) ppo_prof_end(slot, st, 2.0 * B * (400.0 * 32 * 256 + 81.0 * 64 * 512 + 49.0 * 32 * 576));
  PPO_LAUNCH_CHECK("trunk_fwd_kernel");
  return 0;
}

// CNNBase fc (model.py:181): out[m * ldo + n] = relu(x [M][1568] · W4p [H][1568]^T + b), W4p the packed
// segment of ppo_pack_weights (its bf16 planes follow it)
PPO_API int ppo_fc_fwd(const float* x, int M, const float* w4p, const float* b, int H, float* out, int ldo,
                       void* stream) {
  PPO_REQUIRE(H > 0 && H % 8 == 0 && ldo >= H, "ppo_fc_fwd: H=%d ldo=%d", H, ldo);
  const int K = 1568;
  if (M > 0 && M <= g_small_b) return small_linear_fwd(x, nullptr, M, K, K, w4p, b, H, out, ldo, 1, as_stream(stream));
  if (use_x9()) {
    // tiles dealt n-fastest per XCD (igemm_x9.h tile_of); rollout-sized M (4096 rows)
    // fills a quarter of the chip with 128 x 128 tiles: 8 waves of 16 x 64 there
    // (0.060 vs 0.070 ms for 128 x 64)
    const bool wide = ((M + 127LL) / 128) * ((H + 127) / 128) >= 2LL * device_cus();
    const bool abuf = 4LL * M * K < 0x80000000LL;   // DenseReluFwdB's 32-bit offsets
#define PPO_FC(T, CFG)                                                                               \
  {                                                                                                  \
    T<CFG> p;                                                                                        \
    p.x = x; p.w = w4p; p.bias = b; p.out = out; p.M = M; p.N = H; p.K = K; p.ldo = ldo; p.relu = 1; \
    set_planes(p, w4p, (long long)H * K, H, K);                                                      \
    p.n_fast = 1;                                                                                    \
    p.vec = H % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)out & 15) == 0 &&                              \
            (b == nullptr || ((uintptr_t)b & 15) == 0);                                              \
    return launch_x9(p, M, H, 1, as_stream(stream), "fc_fwd", 2.0 * M * H * K);                      \
  }
    if (wide && abuf) PPO_FC(DenseReluFwdB, XP128)   // 0.546-0.551 ms; 8 waves of 16 x 128 0.563-0.565 (r05_v_fc_fwd_tiles_kbench.log)
    if (wide) PPO_FC(DenseReluFwd, XP128)
    if (abuf) PPO_FC(DenseReluFwdB, XP128x64w8)
    PPO_FC(DenseReluFwd, XP128x64w8)
#undef PPO_FC
  }
  DenseReluFwd<CfgN128> p;
  p.x = x; p.w = w4p; p.bias = b; p.out = out; p.M = M; p.N = H; p.K = K; p.ldo = ldo; p.relu = 1;
  return launch(p, M, H, 1, as_stream(stream), "fc_fwd", 2.0 * M * H * K);
}

// Split-K fc forward for rollout-sized M (4,096 rows): 49 k-steps of one 128 x 64 tile
// per CU are latency-bound (0.28 of the MFMA roofline); Z K-slices run Z blocks per
// tile (two resident per CU), their partials go to the caller's workspace slab
// [Z][M][H] and fc_splitk_reduce_kernel sums them in a fixed order, adds the bias
// and applies ReLU.
template <class C_>
struct DenseFwdSplitK : DenseReluFwdB<C_> {   // branch-free operand loads (the launcher checks 4·M·K < 2^31)
  float* slab = nullptr;
  int chunk = 0;   // k per slice, a multiple of 32
  __device__ void k_range(int z, int& b, int& e) const {
    b = z * chunk < this->K ? z * chunk : this->K;
    e = b + chunk < this->K ? b + chunk : this->K;
  }
  __device__ void store(int m, int n, int z, float v) const {
    if (m < this->M && n < this->N) slab[((size_t)z * this->M + m) * this->N + n] = v;
  }
  // vec = 1 (16-B slab rows): the raw partials of columns n .. n + 3 (no bias, no ReLU)
  __device__ void store4(int m, int n, int z, const f32x4& v) const {
    if (m < this->M && n < this->N) *reinterpret_cast<f32x4*>(slab + ((size_t)z * this->M + m) * this->N + n) = v;
  }
};


__global__ __launch_bounds__(256) void fc_splitk_reduce_kernel(const float* __restrict__ slab, int Z, int M, int N,
                                                               const float* __restrict__ bias, float* __restrict__ out,
                                                               int ldo) {
  const int n4 = N >> 2;
  const long long total = (long long)M * n4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int m = (int)(i / n4), q = (int)(i - (long long)m * n4);
    const f32x4* src = reinterpret_cast<const f32x4*>(slab + (size_t)m * N) + q;
    f32x4 v = src[0];
    for (int z = 1; z < Z; ++z) v += src[(size_t)z * M * n4];
    const f32x4 b = reinterpret_cast<const f32x4*>(bias)[q];
    f32x4 y;
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = fmaxf(v[r] + b[r], 0.f);
    *reinterpret_cast<f32x4*>(out + (size_t)m * ldo + 4 * q) = y;
  }
}

// ppo_fc_fwd with a caller-owned workspace (ws, ws_bytes): rollout-sized M takes the
// split-K form when ws holds its slab (ppo_fc_fwd_ws_bytes), else ppo_fc_fwd
PPO_API long long ppo_fc_fwd_ws_bytes(int M, int H) {
  const int Z = g_tune[TK_FC_SPLITK];
  if (Z <= 1 || M <= g_small_b || (long long)M * H > 4096LL * 1024) return 0;
  return 4LL * Z * M * H;
}

PPO_API int ppo_fc_fwd_ws(const float* x, int M, const float* w4p, const float* b, int H, float* out, int ldo,
                          float* ws, long long ws_bytes, void* stream) {
  const long long need = ppo_fc_fwd_ws_bytes(M, H);
  if (!use_x9() || need == 0 || ws == nullptr || ws_bytes < need || ldo % 4 != 0 || H % 4 != 0 || 4LL * M * 1568 >= 0x80000000LL ||
      ((uintptr_t)out & 15) != 0 || ((uintptr_t)ws & 15) != 0 || ((uintptr_t)b & 15) != 0)
    return ppo_fc_fwd(x, M, w4p, b, H, out, ldo, stream);
  const int K = 1568, Z = (int)(need / (4LL * M * H));
  hipStream_t st = as_stream(stream);
  int rc;
#define PPO_FCSK(CFG, VEC)                                                                   \
  {                                                                                          \
    DenseFwdSplitK<CFG> p;                                                                   \
    p.x = x; p.w = w4p; p.bias = b; p.out = out; p.M = M; p.N = H; p.K = K; p.ldo = ldo; p.relu = 1; \
    set_planes(p, w4p, (long long)H * K, H, K);                                              \
    p.n_fast = 1;                                                                            \
    p.slab = ws;                                                                             \
    p.vec = VEC;                                                                             \
    p.chunk = ((K + Z - 1) / Z + 31) / 32 * 32;                                              \
    rc = launch_x9(p, M, H, Z, st, "fc_fwd", 2.0 * M * H * K);                               \
  }
  if (g_tune[TK_FC_SPLITK_TILE]) PPO_FCSK(XP128, 1)
  else PPO_FCSK(XP128x64w8, 0)
#undef PPO_FCSK
  if (rc) return rc;
  const long long n = (long long)M * (H / 4);
  fc_splitk_reduce_kernel<<<(unsigned)std::min<long long>((n + 255) / 256, 4096), 256, 0, st>>>(ws, Z, M, H, b, out,
                                                                                               ldo);
  PPO_LAUNCH_CHECK("fc_splitk_reduce_kernel");
  return 0;
}

// Linear + ReLU: out [M][N] = relu(x [M][K] · w [N][K]^T + b)
PPO_API int ppo_linear_relu_fwd(const float* x, int M, int K, const float* w, const float* b, int N, float* out,
                                void* stream) {
  PPO_REQUIRE(K % 4 == 0, "ppo_linear_relu_fwd: K=%d must be a multiple of 4", K);
  if (M > 0 && M <= g_small_b) return small_linear_fwd(x, nullptr, M, K, K, w, b, N, out, N, 1, as_stream(stream));
  if (use_x9()) {
    DenseReluFwd<X128> p;
    p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K;
    return launch_x9(p, M, N, 1, as_stream(stream), "linear_relu_fwd", 2.0 * M * N * K);
  }
  if (N % 128 == 0) {
    DenseReluFwd<CfgN128> p;
    p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K;
    return launch(p, M, N, 1, as_stream(stream), "linear_relu_fwd", 2.0 * M * N * K);
  }
  DenseReluFwd<CfgN64> p;
  p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K;
  return launch(p, M, N, 1, as_stream(stream), "linear_relu_fwd", 2.0 * M * N * K);
}

// Linear with row strides: out[m*ldo + n] = act(x[idx(m)*lda + k] · w[n][k] + b[n]); b, idx may be NULL;
// act 0 none, 1 ReLU, 2 tanh
PPO_API int ppo_linear_fwd_ex(const float* x, const int64_t* idx, int M, int K, int lda, const float* w, const float* b,
                              int N, float* out, int ldo, int act, void* stream) {
  PPO_REQUIRE(K % 4 == 0 && lda % 4 == 0, "ppo_linear_fwd_ex: K=%d lda=%d must be multiples of 4", K, lda);
  PPO_REQUIRE(act >= 0 && act <= 2, "ppo_linear_fwd_ex: act=%d", act);
  if (M > 0 && M <= g_small_b) return small_linear_fwd(x, idx, M, K, lda, w, b, N, out, ldo, act, as_stream(stream));
  if (use_x9()) {
    if (N <= 64) {
      DenseReluFwd<X64> p;
      p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldo = ldo; p.relu = act;
      p.idx = idx;
      return launch_x9(p, M, N, 1, as_stream(stream), "linear_fwd_ex", 2.0 * M * N * K);
    }
#define PPO_LEX(CFG)                                                                                       \
  {                                                                                                        \
    DenseReluFwd<CFG> p;                                                                                   \
    p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldo = ldo; p.relu = act; \
    p.idx = idx;                                                                                           \
    p.vec = N % 4 == 0 && (ldo ? ldo : N) % 4 == 0 && ((uintptr_t)out & 15) == 0 &&                        \
            (b == nullptr || ((uintptr_t)b & 15) == 0);                                                    \
    return launch_x9(p, M, N, 1, as_stream(stream), "linear_fwd_ex", 2.0 * M * N * K);                     \
  }
    // rollout-sized M (the GRU input projection at 4,096 rows: 192 tiles of 128 x 128 for
    // 256 CUs) takes 64 x 64 tiles
    // 0.024 vs 0.028-0.031 ms at 4,096 x 272 x 768 (profiles/r05_m_gi.log)
    if (((M + 127LL) / 128) * ((N + 127) / 128) < 2LL * device_cus()) PPO_LEX(X64s)
    PPO_LEX(X128)
#undef PPO_LEX
  }
  if (N % 128 == 0) {
    DenseReluFwd<CfgN128> p;
    p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldo = ldo; p.relu = act;
    p.idx = idx;
    return launch(p, M, N, 1, as_stream(stream), "linear_fwd_ex", 2.0 * M * N * K);
  }
  DenseReluFwd<CfgN64> p;
  p.x = x; p.w = w; p.bias = b; p.out = out; p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldo = ldo; p.relu = act;
  p.idx = idx;
  return launch(p, M, N, 1, as_stream(stream), "linear_fwd_ex", 2.0 * M * N * K);
}

// dx [M][N] = g(act) * (dy [M][K] · wt [N][K]^T); act row stride ldact (act NULL: no mask);
// mode 1: g = [act > 0] (ReLU), 2: g = 1 - act² (tanh)
PPO_API int ppo_linear_dgrad_ex(const float* dy, int M, int K, const float* wt, int N, const float* act, int ldact,
                                int mode, float* dx, void* stream) {
  PPO_REQUIRE(K % 4 == 0, "ppo_linear_dgrad_ex: K=%d must be a multiple of 4", K);
  if (use_x9()) {
    DenseDgradMask<X128> p;
    p.dy = dy; p.wt = wt; p.act = act; p.dx = dx; p.M = M; p.N = N; p.K = K; p.ldact = ldact; p.mode = mode;
    p.vec = N % 4 == 0 && (ldact ? ldact : N) % 4 == 0 && ((uintptr_t)dx & 15) == 0 &&
            (act == nullptr || ((uintptr_t)act & 15) == 0);
    return launch_x9(p, M, N, 1, as_stream(stream), "linear_dgrad_ex", 2.0 * M * N * K);
  }
  DenseDgradMask<CfgN128> p;
  p.dy = dy; p.wt = wt; p.act = act; p.dx = dx; p.M = M; p.N = N; p.K = K; p.ldact = ldact; p.mode = mode;
  return launch(p, M, N, 1, as_stream(stream), "linear_dgrad_ex", 2.0 * M * N * K);
}

__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ src, int rows, int cols,
                                                        float* __restrict__ dst) {
  const long long total = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i / rows), r = (int)(i - (long long)c * rows);
    dst[i] = src[(size_t)r * cols + c];
  }
}

// dst [cols][rows] = src [rows][cols]ᵀ (weight transposes for dgrad B operands)
PPO_API int ppo_transpose(const float* src, int rows, int cols, float* dst, void* stream) {
  PPO_REQUIRE(rows > 0 && cols > 0, "ppo_transpose: %d x %d", rows, cols);
  long long b = ((long long)rows * cols + 255) / 256;
  transpose_kernel<<<(unsigned)(b < 2048 ? b : 2048), 256, 0, as_stream(stream)>>>(src, rows, cols, dst);
  PPO_LAUNCH_CHECK("transpose_kernel");
  return 0;
}

// dx [M][N] = (act > 0) * (dy [M][K] · wt [N][K]^T)
PPO_API int ppo_linear_dgrad_mask(const float* dy, int M, int K, const float* wt, int N, const float* act, float* dx,
                                  void* stream) {
  PPO_REQUIRE(K % 4 == 0, "ppo_linear_dgrad_mask: K=%d must be a multiple of 4", K);
  if (use_x9()) {   // wt = the packed W4T segment [1568][H] (planes follow); 8 waves of 16 x 128:
    PPO_REQUIRE(K % 8 == 0, "ppo_linear_dgrad_mask: K=%d must be a multiple of 8", K);   // 0.75 vs 0.87 ms (4 waves)
#define PPO_DGM(T)                                                                                          \
  {                                                                                                         \
    T<XP128w8> p;                                                                                           \
    p.dy = dy; p.wt = wt; p.act = act; p.dx = dx; p.M = M; p.N = N; p.K = K;                                \
    set_planes(p, wt, (long long)N * K, N, K);                                                              \
    p.n_fast = 0;   /* m fastest: the 134 MB dy fits the Infinity Cache, the weight tile stays L2-resident */ \
    p.vec = N % 4 == 0 && ((uintptr_t)dx & 15) == 0 && (act == nullptr || ((uintptr_t)act & 15) == 0);     \
    return launch_x9(p, M, N, 1, as_stream(stream), "linear_dgrad_mask", 2.0 * M * N * K);                  \
  }
    if (4LL * M * K < 0x80000000LL) PPO_DGM(DenseDgradMaskB)   // 32-bit buffer offsets
    PPO_DGM(DenseDgradMask)
#undef PPO_DGM
  }
  DenseDgradMask<CfgN128> p;
  p.dy = dy; p.wt = wt; p.act = act; p.dx = dx; p.M = M; p.N = N; p.K = K;
  return launch(p, M, N, 1, as_stream(stream), "linear_dgrad_mask", 2.0 * M * N * K);
}

// The fc dgrad with conv3's ReLU mask as bits (ppo_conv3_fwd_mask: uint16 [M][49][2],
// bit j of word (p, t) = feature 32 p + 16 t + j): 196 B per row read in the epilogue
// instead of the 6,272 B fp32 activation (0.605 vs 0.695 ms for the fc dgrad at the c3
// minibatch with no mask read at all, profiles/r06_s8_fc_dgrad_mask_kbench.log)
template <class Base>
struct WithMask3Bits : Base {
  const uint16_t* mbits = nullptr;
  __device__ uint32_t bits(int m, int n) const { return (uint32_t)mbits[(size_t)m * 98 + (n >> 4)] >> (n & 15); }
  __device__ void store(int m, int n, int, float v) const {
    if (m < this->M && n < this->N) this->dx[(size_t)m * this->N + n] = (bits(m, n) & 1u) ? v : 0.f;
  }
  __device__ void store4(int m, int n, int, const f32x4& v) const {
    if (m >= this->M || n >= this->N) return;
    const uint32_t b = bits(m, n);
    f32x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = ((b >> r) & 1u) ? v[r] : 0.f;
    *reinterpret_cast<f32x4*>(this->dx + (size_t)m * this->N + n) = o;
  }
};

PPO_API int ppo_fc_dgrad_bits(const float* dy, int M, int K, const float* wt, const uint16_t* mbits, float* dx,
                              void* stream) {
  PPO_REQUIRE(M >= 0 && K > 0 && K % 8 == 0 && mbits != nullptr, "ppo_fc_dgrad_bits: M=%d K=%d", M, K);
  const int N = 1568;
  if (use_x9() && 4LL * M * K < 0x80000000LL) {   // as ppo_linear_dgrad_mask (wt: the packed W4T segment)
    WithMask3Bits<DenseDgradMaskB<XP128w8>> p;
    p.dy = dy; p.wt = wt; p.act = nullptr; p.dx = dx; p.M = M; p.N = N; p.K = K; p.mbits = mbits;
    set_planes(p, wt, (long long)N * K, N, K);
    p.n_fast = 0;
    p.vec = ((uintptr_t)dx & 15) == 0;
    return launch_x9(p, M, N, 1, as_stream(stream), "linear_dgrad_mask", 2.0 * M * N * K);
  }
  WithMask3Bits<DenseDgradMask<CfgN128>> p;
  p.dy = dy; p.wt = wt; p.act = nullptr; p.dx = dx; p.M = M; p.N = N; p.K = K; p.mbits = mbits;
  return launch(p, M, N, 1, as_stream(stream), "linear_dgrad_mask", 2.0 * M * N * K);
}

template <bool BITS>
static int conv3_dgrad_img(const float* dz3, int B, const float* w3d, const float* mask, float* dz2, void* stream) {
  if (B <= 0) return 0;
  const unsigned nb = img_grid(B);
  int slot;
  const bool prof = ppo_prof_begin("conv3_dgrad", as_stream(stream), &slot);
  const uint16_t* wpl = planes_of(w3d, 64 * 288);
  if (g_products == 9) conv3_dgrad_x9_kernel<9, BITS><<<nb, 512, 0, as_stream(stream)>>>(dz3, B, wpl, mask, dz2, g_stagger);
  else if (g_products == 1) conv3_dgrad_x9_kernel<1, BITS><<<nb, 512, 0, as_stream(stream)>>>(dz3, B, wpl, mask, dz2, g_stagger);
  else conv3_dgrad_x9_kernel<6, BITS><<<nb, 512, 0, as_stream(stream)>>>(dz3, B, wpl, mask, dz2, g_stagger);
  if (prof) ppo_prof_end(slot, as_stream(stream), 2.0 * B * 49 * 32 * 576);
  PPO_LAUNCH_CHECK("conv3_dgrad_x9_kernel");
  return 0;
}

// conv3 dgrad with conv2's ReLU mask as bits (m2bits [B][81] u64 from ppo_conv2_fwd_mask)
PPO_API int ppo_conv3_dgrad_bits_ok() { return 1; }
PPO_API int ppo_conv3_dgrad_bits(const float* dz3, int B, const float* w3d, const uint64_t* m2bits, float* dz2,
                                 void* stream) {
  PPO_REQUIRE(m2bits != nullptr, "ppo_conv3_dgrad_bits: null mask");
  return conv3_dgrad_img<true>(dz3, B, w3d, reinterpret_cast<const float*>(m2bits), dz2, stream);
}

PPO_API int ppo_conv3_dgrad(const float* dz3, int B, const float* w3d, const float* a2, float* dz2, void* stream) {
  return conv3_dgrad_img<false>(dz3, B, w3d, a2, dz2, stream);
}

template <bool BITS>
static int conv2_dgrad_img(const float* dz2, int B, const float* w2d, const float* mask, float* dz1, void* stream) {
  if (B <= 0) return 0;
  const unsigned nb = img_grid(B);
  int slot;
  const bool prof = ppo_prof_begin("conv2_dgrad", as_stream(stream), &slot);
  const uint16_t* wpl = planes_of(w2d, 128 * 256);
  const int sg = g_stagger & ~2;
  if (g_products == 9) conv2_dgrad_x9_kernel<9, BITS><<<nb, 512, 0, as_stream(stream)>>>(dz2, B, wpl, mask, dz1, sg);
  else if (g_products == 1) conv2_dgrad_x9_kernel<1, BITS><<<nb, 512, 0, as_stream(stream)>>>(dz2, B, wpl, mask, dz1, sg);
  else conv2_dgrad_x9_kernel<6, BITS><<<nb, 512, 0, as_stream(stream)>>>(dz2, B, wpl, mask, dz1, sg);
  if (prof) ppo_prof_end(slot, as_stream(stream), 2.0 * B * 81 * 64 * 512);
  PPO_LAUNCH_CHECK("conv2_dgrad_x9_kernel");
  return 0;
}

// conv2 dgrad with the conv1 ReLU mask as bits (m1bits [B][400] u32 from ppo_conv1_fwd_mask)
PPO_API int ppo_conv2_dgrad_bits_ok() { return 1; }
PPO_API int ppo_conv2_dgrad_bits(const float* dz2, int B, const float* w2d, const uint32_t* m1bits, float* dz1,
                                 void* stream) {
  PPO_REQUIRE(m1bits != nullptr, "ppo_conv2_dgrad_bits: null mask");
  return conv2_dgrad_img<true>(dz2, B, w2d, reinterpret_cast<const float*>(m1bits), dz1, stream);
}

PPO_API int ppo_conv2_dgrad(const float* dz2, int B, const float* w2d, const float* a1, float* dz1, void* stream) {
  return conv2_dgrad_img<false>(dz2, B, w2d, a1, dz1, stream);
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

// chunks are multiples of 32 rows: whole k-tiles of both cores (BK 16 and 32)
static inline int wgrad_chunk(long long R, int Z) {
  long long kt = (R + 31) / 32;
  return (int)(((kt + Z - 1) / Z) * 32);
}

template <class P>
static void set_wgrad(P& p, const float* dz, int COUT, long long R, int Z, float* slab, float* slab_bias, int NW) {
  p.dz = dz; p.COUT = COUT; p.R = R; p.chunk = wgrad_chunk(R, Z); p.slab = slab; p.slab_bias = slab_bias; p.NW = NW;
}

using CfgW32 = Cfg<32, 256, 1, 4, false, false, true>;
using CfgWfc = Cfg<128, 128, 2, 2, false, false, true>;

// conv1 wgrad partials: slab [Z][32][C*64], slab_bias [Z][32]
PPO_API int ppo_conv1_wgrad(const float* dz1, const void* obs, int obs_is_u8, const int64_t* idx, long long row0,
                            int C, int B, int Z, float* slab, float* slab_bias, void* stream) {
  const long long R = (long long)B * 400;
  PPO_REQUIRE(R < 0x7fffffffLL, "ppo_conv1_wgrad: B too large");
  const double fl = 2.0 * R * 32 * C * 64;
  // u8 rows, C = 4: the k-split kernels (conv1w.hip, tunes 8-10, fp32 dz) or the
  // part-pipelined kernel (tune 5; the half-precision mode's, bf16 dz)
  if (obs_is_u8 && C == 4 && (g_tune[TK_CONV1_WGRAD] == 5 || g_products == 1)) {
    if (B <= 0 || Z <= 0) return 0;
    PPO_REQUIRE((B + Z - 1) / Z <= 512, "ppo_conv1_wgrad: %d images over %d blocks (at most 512 per block)", B, Z);
    int slot;
    const bool prof = ppo_prof_begin("conv1_wgrad_u8", as_stream(stream), &slot);
    if (g_products == 1)
      conv1_wgrad_parts_kernel<1, 16, 2><<<Z, 1024, 0, as_stream(stream)>>>(dz1, (const uint8_t*)obs, idx, row0, B,
                                                                            slab, slab_bias, 0);
    else
      conv1_wgrad_parts_kernel<3, 16, 2><<<Z, 1024, 0, as_stream(stream)>>>(dz1, (const uint8_t*)obs, idx, row0, B,
                                                                            slab, slab_bias, g_stagger >> 4);
    if (prof) ppo_prof_end(slot, as_stream(stream), fl);
    PPO_LAUNCH_CHECK("conv1_wgrad_parts_kernel");
    return 0;
  }
  if (obs_is_u8 && C == 4)
    return g_tune[TK_CONV1_WGRAD] >= 9
               ? conv1_wgrad_kw3(dz1, (const uint8_t*)obs, idx, row0, B, Z, slab, slab_bias, stream,
                                 g_tune[TK_CONV1_WGRAD] == 10 ? 8 : 4)
               : conv1_wgrad_kw(dz1, (const uint8_t*)obs, idx, row0, B, Z, slab, slab_bias, stream);
  if (!obs_is_u8 && C == 4 && ((uintptr_t)obs & 15) == 0)   // conv1f.hip
    return ppo_conv1_wgrad_f32(dz1, (const float*)obs, idx, row0, B, Z, slab, slab_bias, stream);
  if (obs_is_u8) {   // any other channel count: the generic fp32-MFMA tile GEMM
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
  if (B <= 0 || Z <= 0) return 0;
  int slot;
  const bool prof = ppo_prof_begin("conv2_wgrad", as_stream(stream), &slot);
  PPO_LAUNCH_NP(conv2_wgrad_x9_kernel, Z, 512, as_stream(stream), dz2, a1, B, slab, slab_bias);
  if (prof) ppo_prof_end(slot, as_stream(stream), 2.0 * B * 81 * 64 * 512);
  PPO_LAUNCH_CHECK("conv2_wgrad_x9_kernel");
  return 0;
}

PPO_API int ppo_conv3_wgrad(const float* dz3, const float* a2, int B, int Z, float* slab, float* slab_bias,
                            void* stream) {
  if (B <= 0 || Z <= 0) return 0;
  int slot;
  const bool prof = ppo_prof_begin("conv3_wgrad", as_stream(stream), &slot);
  PPO_LAUNCH_NP(conv3_wgrad_x9_kernel, Z, 768, as_stream(stream), dz3, a2, B, slab, slab_bias);
  if (prof) ppo_prof_end(slot, as_stream(stream), 2.0 * B * 49 * 32 * 576);
  PPO_LAUNCH_CHECK("conv3_wgrad_x9_kernel");
  return 0;
}

// dW[n][k] = Σ_r dy[r][n] x[r][k]: slab [Z][N][K], slab_bias [Z][N]
PPO_API int ppo_linear_wgrad(const float* dy, const float* x, int R, int N, int K, int Z, float* slab,
                             float* slab_bias, void* stream) {
  PPO_REQUIRE(N % 4 == 0 && K % 4 == 0, "ppo_linear_wgrad: N=%d K=%d must be multiples of 4", N, K);
  // split path: the fc layer (N >= 128) whenever the split core is on (0.82 vs
  // 1.03 ms at the c3 minibatch); the narrow GRU/MLP layers only with x9 = 2
  if (use_x9_all() || (use_x9() && N >= 128)) {
    if (N <= 64) {
      DenseWgrad<XW64> p;
      set_wgrad(p, dy, N, R, Z, slab, slab_bias, K);
      p.x = x; p.K = K;
      return launch_x9(p, N, K, Z, as_stream(stream), "linear_wgrad", 2.0 * R * N * K);
    }
    // split at staging, 256 x 128 tiles: 0.727 vs 0.775 ms (in-loop split) at the c3 minibatch;
    // branch-free buffer loads where the operands fit 31-bit offsets
    if ((long long)R * (N > K ? N : K) * 4 < 0x7fffffffLL) {
      DenseWgradB<SW256x128> p;
      set_wgrad(p, dy, N, R, Z, slab, slab_bias, K);
      p.x = x; p.K = K; p.n_fast = 0;
      p.vec = K % 4 == 0 && ((uintptr_t)slab & 15) == 0;
      return launch_x9(p, N, K, Z, as_stream(stream), "linear_wgrad", 2.0 * R * N * K);
    }
    DenseWgrad<SW256x128> p;
    set_wgrad(p, dy, N, R, Z, slab, slab_bias, K);
    p.x = x; p.K = K; p.n_fast = 0;
    p.vec = K % 4 == 0 && ((uintptr_t)slab & 15) == 0;
    return launch_x9(p, N, K, Z, as_stream(stream), "linear_wgrad", 2.0 * R * N * K);
  }
  DenseWgrad<CfgWfc> p;
  set_wgrad(p, dy, N, R, Z, slab, slab_bias, K);
  p.x = x; p.K = K;
  return launch(p, N, K, Z, as_stream(stream), "linear_wgrad", 2.0 * R * N * K);
}

// Σ over the Z split partials (fixed order) -> gw (torch order, see ColMap) and gb
PPO_API int ppo_wgrad_reduce(const float* slab, const float* slab_bias, int Z, int M, int NW, int kind, int a, int b,
                             float* gw, float* gb, float scale, int accumulate, void* stream) {
  PPO_REQUIRE(kind >= 0 && kind <= 3, "ppo_wgrad_reduce: kind=%d", kind);
  ProfScope prof("wgrad_reduce", as_stream(stream), 4.0 * (double)Z * M * (NW + 1) + 4.0 * M * (NW + 1));
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
