// Small-batch forward path (batch-1 evaluation act,
// T/run_evaluation.py:25-122 -> Policy.act on one env).  At a handful of
// images the image-resident persistent kernels and the tile GEMMs run one or
// two workgroups each, serially through their k loops (fc 1568 -> H: 48 us at
// B = 1, measured); here every output element gets its own thread (convs) or
// wave (linears) and the whole chip works on one sample.  Plain fp32 FMAs in a
// fixed order per element: exact fp32 arithmetic like the reference's CPU
// path (model.py:169-199 convs, Linear), deterministic.  Dispatched by the
// forward entry points in gemm.hip when B <= ppo_tune_get("small_b").
#include "common.h"
#include "small.h"

namespace {
constexpr int IMG = 84, IMG2 = 84 * 84;

__device__ __forceinline__ long long sample_row(const int64_t* idx, long long row0, int b) {
  return idx ? (long long)idx[b] : row0 + b;
}

// conv1 (8x8 stride 4, C channels of the NCHW observation, torch weight layout
// [32][C][8][8]) -> NHWC [B][20][20][32]; u8 observations: Σ u·w scaled by
// 1/255 before the bias (as the MFMA kernels' epilogue).  A group of G >= C lanes
// per output (b, px, co), lane c < C summing channel c's 8x8 window; the partials
// are combined in a fixed order (c ascending) through shuffles.
template <typename InT, int G>
__global__ __launch_bounds__(256) void small_conv1_kernel(const InT* __restrict__ obs,
                                                          const int64_t* __restrict__ idx, long long row0, int C,
                                                          int B, const float* __restrict__ w1,
                                                          const float* __restrict__ b1, float* __restrict__ out) {
  static_assert(G >= 1 && G <= 8 && (64 % G) == 0, "channel group");
  const int t = blockIdx.x * 256 + threadIdx.x, c = t % G, o = t / G;
  const bool on = o < B * 400 * 32;
  const int oo = on ? o : 0, cc = c < C ? c : 0;
  const int co = oo & 31, bp = oo >> 5, b = bp / 400, p = bp - b * 400, oy = p / 20, ox = p - oy * 20;
  const InT* src = obs + sample_row(idx, row0, b) * (long long)(C * IMG2) + cc * IMG2 + (4 * oy) * IMG + 4 * ox;
  const float* wr = w1 + (co * C + cc) * 64;
  float acc = 0.f;
#pragma unroll
  for (int ky = 0; ky < 8; ++ky) {
    float v[8];
    if constexpr (sizeof(InT) == 1) {
      const uint32_t* r = reinterpret_cast<const uint32_t*>(src + ky * IMG);
      const uint32_t u0 = r[0], u1 = r[1];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = (float)((u0 >> (8 * i)) & 255u);
        v[4 + i] = (float)((u1 >> (8 * i)) & 255u);
      }
    } else {
      const f32x4* r = reinterpret_cast<const f32x4*>(src + ky * IMG);
      const f32x4 a = r[0], bq = r[1];
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
      v[4] = bq[0]; v[5] = bq[1]; v[6] = bq[2]; v[7] = bq[3];
    }
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(wr + 8 * ky), w1v = *reinterpret_cast<const f32x4*>(wr + 8 * ky + 4);
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) acc = fmaf(v[kx], w0[kx], acc);
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) acc = fmaf(v[4 + kx], w1v[kx], acc);
  }
  if (c >= C) acc = 0.f;
  // fixed-order combine of the channel partials: lane c = 0 gathers c = 1 .. G-1
  float tot = acc;
#pragma unroll
  for (int j = 1; j < G; ++j) tot += __shfl_down(acc, j, 64);
  if (on && c == 0) {
    if constexpr (sizeof(InT) == 1) tot *= (1.0f / 255.0f);
    out[(size_t)bp * 32 + co] = fmaxf(tot + b1[co], 0.f);
  }
}

// NHWC conv + bias + ReLU with weights packed [COUT][K], k = (ky, kx, ci)
// (ppo_pack_weights' fp32 segment).  A group of 16 lanes per output (b, output
// pixel, co): lane l sums the float4 chunks l, l + 16, ... of K (consecutive
// lanes read consecutive channels: coalesced), then a fixed-order butterfly.
template <int HIN, int CIN, int KS, int ST, int HOUT, int COUT>
__global__ __launch_bounds__(256) void small_conv_kernel(const float* __restrict__ in, int B,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias, float* __restrict__ out) {
  constexpr int P = HOUT * HOUT, K = KS * KS * CIN, NC = K / 4, L = 16;
  static_assert(CIN % 4 == 0, "float4 channel groups");
  const int t = blockIdx.x * 256 + threadIdx.x, l = t & (L - 1), o = t / L;
  const bool on = o < B * P * COUT;
  const int oo = on ? o : 0;
  const int co = oo % COUT, bp = oo / COUT, b = bp / P, p = bp - b * P, oy = p / HOUT, ox = p - oy * HOUT;
  const float* src = in + ((size_t)(b * HIN + ST * oy) * HIN + ST * ox) * CIN;
  const float* wr = w + (size_t)co * K;
  float acc = 0.f;
#pragma unroll 4
  for (int f = l; f < NC; f += L) {
    const int k = 4 * f, tap = k / CIN, ci = k - tap * CIN, ky = tap / KS, kx = tap - ky * KS;
    const f32x4 av = *reinterpret_cast<const f32x4*>(src + (ky * HIN + kx) * CIN + ci);
    const f32x4 wv = *reinterpret_cast<const f32x4*>(wr + k);
    acc = fmaf(av[0], wv[0], acc);
    acc = fmaf(av[1], wv[1], acc);
    acc = fmaf(av[2], wv[2], acc);
    acc = fmaf(av[3], wv[3], acc);
  }
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, L);
  if (on && l == 0) out[(size_t)bp * COUT + co] = fmaxf(acc + bias[co], 0.f);
}

// out[m * ldo + n] = act(Σ_k x[row(m) * lda + k] · w[n][k] + b[n]); act 0 none,
// 1 ReLU, 2 tanh.  One wave per (m, n): lanes stride k by float4, then a
// butterfly sum (fixed order).
__global__ __launch_bounds__(256) void small_linear_kernel(const float* __restrict__ x,
                                                           const int64_t* __restrict__ idx, int M, int K, int lda,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           int N, float* __restrict__ out, int ldo, int act) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wv >= M * N) return;   // wave-uniform
  const int m = wv / N, n = wv - m * N;
  const float* xr = x + sample_row(idx, 0, m) * (long long)lda;
  const float* wr = w + (size_t)n * K;
  float acc = 0.f;
  for (int k = 4 * lane; k < K; k += 256) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(xr + k), q = *reinterpret_cast<const f32x4*>(wr + k);
    acc = fmaf(a[0], q[0], acc);
    acc = fmaf(a[1], q[1], acc);
    acc = fmaf(a[2], q[2], acc);
    acc = fmaf(a[3], q[3], acc);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (lane == 0) {
    float v = acc + (b ? b[n] : 0.f);
    if (act == 1) v = fmaxf(v, 0.f);
    else if (act == 2) v = tanhf(v);
    out[(size_t)m * ldo + n] = v;
  }
}

inline unsigned nblocks(long long threads) { return (unsigned)((threads + 255) / 256); }
}  // namespace

template <int G>
static void small_conv1_launch(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                               const float* w1, const float* b1, float* out, hipStream_t s) {
  const unsigned nb = nblocks((long long)B * 400 * 32 * G);
  if (obs_is_u8)
    small_conv1_kernel<uint8_t, G><<<nb, 256, 0, s>>>((const uint8_t*)obs, idx, row0, C, B, w1, b1, out);
  else
    small_conv1_kernel<float, G><<<nb, 256, 0, s>>>((const float*)obs, idx, row0, C, B, w1, b1, out);
}

int small_conv1_fwd(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                    const float* w1, const float* b1, float* out, hipStream_t s) {
  if (B <= 0) return 0;
  PPO_REQUIRE(C >= 1 && C <= 8, "small_conv1_fwd: C=%d (1 .. 8 channels)", C);
  PPO_REQUIRE(obs_is_u8 || ((uintptr_t)obs & 15) == 0, "small_conv1_fwd: fp32 observations must be 16-B aligned");
  if (C == 1) small_conv1_launch<1>(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, s);
  else if (C == 2) small_conv1_launch<2>(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, s);
  else if (C <= 4) small_conv1_launch<4>(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, s);
  else small_conv1_launch<8>(obs, obs_is_u8, idx, row0, C, B, w1, b1, out, s);
  PPO_LAUNCH_CHECK("small_conv1_kernel");
  return 0;
}

int small_conv2_fwd(const float* a1, int B, const float* w2p, const float* b2, float* out, hipStream_t s) {
  if (B <= 0) return 0;
  small_conv_kernel<20, 32, 4, 2, 9, 64><<<nblocks((long long)B * 81 * 64 * 16), 256, 0, s>>>(a1, B, w2p, b2, out);
  PPO_LAUNCH_CHECK("small_conv_kernel<conv2>");
  return 0;
}

int small_conv3_fwd(const float* a2, int B, const float* w3p, const float* b3, float* out, hipStream_t s) {
  if (B <= 0) return 0;
  small_conv_kernel<9, 64, 3, 1, 7, 32><<<nblocks((long long)B * 49 * 32 * 16), 256, 0, s>>>(a2, B, w3p, b3, out);
  PPO_LAUNCH_CHECK("small_conv_kernel<conv3>");
  return 0;
}

int small_linear_fwd(const float* x, const int64_t* idx, int M, int K, int lda, const float* w, const float* b,
                     int N, float* out, int ldo, int act, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  const long long waves = (long long)M * N;
  small_linear_kernel<<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(x, idx, M, K, lda, w, b, N, out, ldo, act);
  PPO_LAUNCH_CHECK("small_linear_kernel");
  return 0;
}
