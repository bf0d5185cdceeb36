// GAE-λ / discounted returns (K3) fused with the advantage difference and its
// moment partials (K4).  Compiled with -ffp-contract=off: results are
// bit-identical to the reference CPU path (tests/golden/gae.npz).
//
// Reference: RolloutStorage.compute_returns,
//   ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/storage.py:82-121
// Advantages: algo/ppo.py:35-37.
//
// Layout (HBM): every per-step scalar lives in its own [T(+1)][N] fp32 plane
// (time-major, env-minor — the reference's [T(+1), N, 1] tensors), so lane n of
// a wave reads/writes element n of a row: 256-B coalesced per wave per plane.
//
// One thread owns one env lane and walks time backwards (the recurrence is
// sequential in t).  Loads for U future steps are issued before the dependent
// arithmetic so each wave keeps 3-4·U loads in flight; with ≥16k lanes per
// launch this streams at the HBM rate (bench.py gae roofline).
#include "common.h"

namespace {

constexpr int GAE_THREADS = 256;
#ifndef PPO_GAE_U
#define PPO_GAE_U 64
#endif
#ifndef PPO_GAE_NT
#define PPO_GAE_NT 1
#endif
// streaming planes: nontemporal loads and stores (PPO_GAE_NT 1), stores only (2), or plain (0)
template <class T_>
__device__ __forceinline__ T_ gld(const T_* p) {
  if constexpr (PPO_GAE_NT == 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <class T_>
__device__ __forceinline__ void gst(T_* p, T_ v) {
  if constexpr (PPO_GAE_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
// time steps prefetched per chunk; with nontemporal loads and stores 64 steps run
// 5.15-5.17 TB/s on 1M lanes, 32 steps 5.05-5.07, against 4.79-4.84 for 16 plain
// (16 + nontemporal 4.68-4.86, nontemporal stores only 4.69-4.72; tools/gae_ab.sh,
// profiles/r04_gae_ab.log, r04_gae_ab2.log)
constexpr int GAE_U = PPO_GAE_U;

// Advantage moments as (count, mean, M2) (the reference's
// advantages.mean() / .std(), T/a2c_ppo_acktr/algo/ppo.py:35-37): each thread
// keeps shifted sums Σ(d - k), Σ(d - k)² about its first value k (exact for a
// constant series, stable when the mean is large against the spread), and the
// thread, wave, block, grid and rank results are combined with Chan et al.'s
// pairwise update — always (lower, higher), so the result is deterministic and
// identical on every lane of a butterfly.
struct Mom {
  double n, mean, m2;
};
struct MomAcc {
  double k = 0.0, s = 0.0, q = 0.0, n = 0.0;
  __device__ __forceinline__ void add(double d) {
    if (n == 0.0) k = d;
    const double e = d - k;
    s += e;
    q += e * e;
    n += 1.0;
  }
  __device__ __forceinline__ Mom get() const {
    if (n == 0.0) return {0.0, 0.0, 0.0};
    const double m2 = q - s * (s / n);
    return {n, k + s / n, m2 > 0.0 ? m2 : 0.0};
  }
};
__device__ __forceinline__ Mom mom_merge(const Mom& a, const Mom& b) {
  const double n = a.n + b.n;
  if (b.n == 0.0) return a;
  if (a.n == 0.0) return b;
  const double d = b.mean - a.mean, f = b.n / n;
  return {n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}
__device__ __forceinline__ Mom wave_merge(Mom m) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const Mom p{__shfl_xor(m.n, o, 64), __shfl_xor(m.mean, o, 64), __shfl_xor(m.m2, o, 64)};
    m = (lane & o) ? mom_merge(p, m) : mom_merge(m, p);
  }
  return m;
}
// block result -> partials[3 blk .. +2]; WAVES waves, lds scratch of WAVES Mom
template <int WAVES>
__device__ __forceinline__ void block_moments(const MomAcc& acc, double* __restrict__ partials) {
  __shared__ Mom red[WAVES];
  const Mom w = wave_merge(acc.get());
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    Mom t = red[0];
    for (int i = 1; i < WAVES; ++i) t = mom_merge(t, red[i]);
    partials[3 * blockIdx.x] = t.n;
    partials[3 * blockIdx.x + 1] = t.mean;
    partials[3 * blockIdx.x + 2] = t.m2;
  }
}

template <bool USE_GAE, bool PTL, bool FUSE_ADV>
__global__ __launch_bounds__(GAE_THREADS) void gae_kernel(
    const float* __restrict__ rewards, float* __restrict__ value_preds,
    const float* __restrict__ masks, const float* __restrict__ bad_masks,
    const float* __restrict__ next_value, float* __restrict__ returns,
    float* __restrict__ adv, double* __restrict__ partials, int T, int N, float g, float gl) {
  const int n = blockIdx.x * GAE_THREADS + threadIdx.x;
  MomAcc mom;
  if (n < N) {
    const size_t NN = (size_t)N;
    const float nv = next_value[n];
    float carry;  // gae (USE_GAE) or returns[t+1] (non-GAE)
    float vnext = nv;
    if (USE_GAE) {
      value_preds[(size_t)T * NN + n] = nv;  // storage.py:90/:108
      carry = 0.0f;
    } else {
      returns[(size_t)T * NN + n] = nv;      // storage.py:101/:118
      carry = nv;
    }
    for (int t0 = T - 1; t0 >= 0; t0 -= GAE_U) {
      float rr[GAE_U], vv[GAE_U], mm[GAE_U], bb[GAE_U];
#pragma unroll
      for (int j = 0; j < GAE_U; ++j) {
        const int t = t0 - j;
        if (t >= 0) {
          rr[j] = gld(rewards + (size_t)t * NN + n);
          mm[j] = gld(masks + (size_t)(t + 1) * NN + n);
          vv[j] = (USE_GAE || PTL || FUSE_ADV) ? gld(value_preds + (size_t)t * NN + n) : 0.0f;
          bb[j] = PTL ? gld(bad_masks + (size_t)(t + 1) * NN + n) : 1.0f;
        }
      }
#pragma unroll
      for (int j = 0; j < GAE_U; ++j) {
        const int t = t0 - j;
        if (t >= 0) {
          float out;
          if (USE_GAE) {
            float a = g * vnext;               // gamma * value_preds[t+1]
            a = a * mm[j];                     //   * masks[t+1]
            float delta = rr[j] + a;           // rewards[t] + ...
            delta = delta - vv[j];             //   - value_preds[t]
            float b = gl * mm[j];              // (gamma*gae_lambda) * masks[t+1]
            b = b * carry;                     //   * gae
            carry = delta + b;
            if (PTL) carry = carry * bb[j];    // gae * bad_masks[t+1]
            out = carry + vv[j];               // returns[t] = gae + value_preds[t]
            vnext = vv[j];
          } else {
            float x = carry * g;               // returns[t+1] * gamma
            x = x * mm[j];                     //   * masks[t+1]
            x = x + rr[j];                     //   + rewards[t]
            if (PTL) {
              x = x * bb[j];
              float keep = 1.0f - bb[j];
              keep = keep * vv[j];
              x = x + keep;
            }
            out = x;
            carry = x;
          }
          gst(returns + (size_t)t * NN + n, out);
          if (FUSE_ADV) {
            const float d = out - vv[j];       // returns[:-1] - value_preds[:-1]
            gst(adv + (size_t)t * NN + n, d);
            mom.add((double)d);
          }
        }
      }
    }
  }
  if (FUSE_ADV) block_moments<GAE_THREADS / 64>(mom, partials);
}

// ---------------------------------------------------------------------------
// Time-parallel mode (tolerance, not bit-exact): for few lanes (c1: 8, c2: 1024)
// the lane-sequential kernel above occupies 1-4 CUs for T dependent steps.  The
// recurrence is affine in the carry,
//   GAE:      g_t   = (δ_t + (γλ·m_{t+1})·g_{t+1})·bm_{t+1}      ret_t = g_t + v_t
//   returns:  ret_t = (γ·m_{t+1}·ret_{t+1} + r_t)·bm_{t+1} + (1 − bm_{t+1})·v_t
// i.e. x_t = a_t + b_t·x_{t+1}, and affine maps compose:  (A, B) after (a, b)
// = (a + b·A, b·B).  A block holds SCAN_LANES consecutive lanes x SCAN_CH time
// chunks (one thread each; the lanes of a chunk row read 64 contiguous bytes):
//   1. every thread folds its chunk into one map (A_c, B_c)       (T/CH steps)
//   2. the carry entering chunk c is the composition of chunks > c applied to
//      x_T, through LDS                                            (≤ CH-1 steps)
//   3. every thread re-walks its chunk from that carry and writes returns (+ adv
//      and its moment partials).
// Only the association of the sums changes: |err| ~ T·ε·max|x| (tests hold it
// to the bit-exact kernel within 2e-6 of max|returns|).
constexpr int SCAN_LANES = 16;
constexpr int SCAN_CH = 16;

template <bool USE_GAE, bool PTL>
__device__ __forceinline__ void gae_affine(const float* __restrict__ rewards, const float* __restrict__ value_preds,
                                           const float* __restrict__ masks, const float* __restrict__ bad_masks,
                                           float nv, size_t NN, int n, int t, int T, float g, float gl, float& a,
                                           float& b, float& v) {
  const float r = rewards[(size_t)t * NN + n];
  const float m = masks[(size_t)(t + 1) * NN + n];
  const float bm = PTL ? bad_masks[(size_t)(t + 1) * NN + n] : 1.0f;
  v = value_preds[(size_t)t * NN + n];
  if (USE_GAE) {
    const float vn = t + 1 < T ? value_preds[(size_t)(t + 1) * NN + n] : nv;
    const float delta = (r + (g * vn) * m) - v;
    a = PTL ? delta * bm : delta;
    b = PTL ? (gl * m) * bm : gl * m;
  } else {
    a = PTL ? r * bm + (1.0f - bm) * v : r;
    b = PTL ? (g * m) * bm : g * m;
  }
}

template <bool USE_GAE, bool PTL, bool FUSE_ADV>
__global__ __launch_bounds__(SCAN_LANES * SCAN_CH) void gae_scan_kernel(
    const float* __restrict__ rewards, float* __restrict__ value_preds, const float* __restrict__ masks,
    const float* __restrict__ bad_masks, const float* __restrict__ next_value, float* __restrict__ returns,
    float* __restrict__ adv, double* __restrict__ partials, int T, int N, float g, float gl) {
  const int l = threadIdx.x % SCAN_LANES, c = threadIdx.x / SCAN_LANES;
  const int n = blockIdx.x * SCAN_LANES + l;
  const int L = (T + SCAN_CH - 1) / SCAN_CH;
  const int t_lo = c * L, t_hi = min(T, t_lo + L);
  const size_t NN = (size_t)N;
  __shared__ float mapA[SCAN_CH][SCAN_LANES], mapB[SCAN_CH][SCAN_LANES];
  const bool live = n < N;
  const float nv = live ? next_value[n] : 0.0f;
  // 1. this chunk's composite map x_{t_lo} = A + B·x_{t_hi}
  float A = 0.0f, B = 1.0f;
  if (live) {
    for (int t = t_hi - 1; t >= t_lo; --t) {
      float a, b, v;
      gae_affine<USE_GAE, PTL>(rewards, value_preds, masks, bad_masks, nv, NN, n, t, T, g, gl, a, b, v);
      A = a + b * A;
      B = b * B;
    }
  }
  mapA[c][l] = A;
  mapB[c][l] = B;
  __syncthreads();
  // 2. carry entering this chunk from above: x_T, then the chunks after this one
  float x = USE_GAE ? 0.0f : nv;
  for (int k = SCAN_CH - 1; k > c; --k) x = mapA[k][l] + mapB[k][l] * x;
  // 3. re-walk with the carry; the storage side effects of the exact kernel
  MomAcc mom;
  if (live) {
    if (t_lo < T && t_hi == T) {   // the last non-empty chunk
      if (USE_GAE) value_preds[(size_t)T * NN + n] = nv;   // storage.py:90/:108
      else returns[(size_t)T * NN + n] = nv;               // storage.py:101/:118
    }
    for (int t = t_hi - 1; t >= t_lo; --t) {
      float a, b, v;
      gae_affine<USE_GAE, PTL>(rewards, value_preds, masks, bad_masks, nv, NN, n, t, T, g, gl, a, b, v);
      x = a + b * x;
      const float out = USE_GAE ? x + v : x;
      returns[(size_t)t * NN + n] = out;
      if (FUSE_ADV) {
        const float d = out - v;
        adv[(size_t)t * NN + n] = d;
        mom.add((double)d);
      }
    }
  }
  if (FUSE_ADV) block_moments<SCAN_LANES * SCAN_CH / 64>(mom, partials);
}

// adv = returns - value_preds over the first T rows, plus moment partials
// (used when storage was modified after compute_returns).
__global__ __launch_bounds__(256) void adv_diff_kernel(const float* __restrict__ returns,
                                                       const float* __restrict__ value_preds,
                                                       float* __restrict__ adv,
                                                       double* __restrict__ partials, long long n) {
  MomAcc mom;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float d = returns[i] - value_preds[i];
    adv[i] = d;
    mom.add((double)d);
  }
  block_moments<4>(mom, partials);
}

// Deterministic fixed-order merge of the block partials -> stats {count, mean, M2}
// (count: the partials' own; the argument is kept for the ABI).
__global__ __launch_bounds__(256) void adv_finalize_kernel(const double* __restrict__ partials, int nparts,
                                                           double count, double* __restrict__ stats) {
  (void)count;
  Mom m{0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < nparts; i += 256) m = mom_merge(m, Mom{partials[3 * i], partials[3 * i + 1],
                                                                       partials[3 * i + 2]});
  __shared__ Mom r[256];
  r[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) r[threadIdx.x] = mom_merge(r[threadIdx.x], r[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[0] = r[0].n;
    stats[1] = r[0].mean;
    stats[2] = r[0].m2;
  }
}

// adv = (adv - mean) / (std + 1e-5) in fp32, from the (possibly rank-merged)
// stats {count, mean, M2}; std is unbiased (torch.std default): sqrt(M2 / (n - 1)).
__global__ __launch_bounds__(256) void adv_normalize_kernel(float* __restrict__ adv, long long n,
                                                            const double* __restrict__ stats) {
  const double cnt = stats[0];
  const double mean = stats[1];
  double var = stats[2] / (cnt - 1.0);
  if (var < 0.0) var = 0.0;
  const float mf = (float)mean;
  const float den = (float)sqrt(var) + 1e-5f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float a = adv[i] - mf;
    adv[i] = a / den;
  }
}

template <bool G, bool P, bool F>
int launch_gae(const float* r, float* v, const float* m, const float* bm, const float* nv, float* ret,
               float* adv, double* partials, int T, int N, float g, float gl, hipStream_t st) {
  gae_kernel<G, P, F><<<ceil_div(N, GAE_THREADS), GAE_THREADS, 0, st>>>(r, v, m, bm, nv, ret, adv, partials,
                                                                       T, N, g, gl);
  PPO_LAUNCH_CHECK("gae_kernel");
  return 0;
}

template <bool G, bool P, bool F>
int launch_gae_scan(const float* r, float* v, const float* m, const float* bm, const float* nv, float* ret,
                    float* adv, double* partials, int T, int N, float g, float gl, hipStream_t st) {
  gae_scan_kernel<G, P, F><<<ceil_div(N, SCAN_LANES), SCAN_LANES * SCAN_CH, 0, st>>>(r, v, m, bm, nv, ret, adv,
                                                                                      partials, T, N, g, gl);
  PPO_LAUNCH_CHECK("gae_scan_kernel");
  return 0;
}

}  // namespace

PPO_API int ppo_gae_partials_count(int N) { return (int)ceil_div(N, GAE_THREADS); }
PPO_API int ppo_gae_scan_partials_count(int N) { return (int)ceil_div(N, SCAN_LANES); }

// Time-parallel compute_returns (same arguments and side effects as
// ppo_compute_returns; partials: 2*ppo_gae_scan_partials_count(N) doubles).
// Within tolerance of the bit-exact kernel, for few lanes / long T.
PPO_API int ppo_compute_returns_scan(const float* rewards, float* value_preds, const float* masks,
                                     const float* bad_masks, const float* next_value, float* returns, float* adv,
                                     double* partials, int T, int N, double gamma, double gae_lambda, int use_gae,
                                     int use_proper_time_limits, void* stream) {
  PPO_REQUIRE(T > 0 && N > 0, "ppo_compute_returns_scan: bad shape T=%d N=%d", T, N);
  PPO_REQUIRE(rewards && value_preds && masks && next_value && returns, "ppo_compute_returns_scan: null pointer");
  PPO_REQUIRE(!use_proper_time_limits || bad_masks, "ppo_compute_returns_scan: bad_masks required");
  PPO_REQUIRE((adv == nullptr) == (partials == nullptr), "ppo_compute_returns_scan: adv and partials go together");
  ProfScope prof("gae_scan", as_stream(stream), (adv ? 20.0 : 16.0) * T * N);
  const float g = (float)gamma;
  const float gl = (float)(gamma * gae_lambda);
  hipStream_t st = as_stream(stream);
  const bool F = adv != nullptr;
#define PPO_SCAN(G_, P_)                                                                                         \
  return F ? launch_gae_scan<G_, P_, true>(rewards, value_preds, masks, bad_masks, next_value, returns, adv,    \
                                          partials, T, N, g, gl, st)                                            \
           : launch_gae_scan<G_, P_, false>(rewards, value_preds, masks, bad_masks, next_value, returns, adv,   \
                                           partials, T, N, g, gl, st);
  if (use_gae) {
    if (use_proper_time_limits) PPO_SCAN(true, true)
    PPO_SCAN(true, false)
  }
  if (use_proper_time_limits) PPO_SCAN(false, true)
  PPO_SCAN(false, false)
#undef PPO_SCAN
}

// storage.py:82-121 (+ ppo.py:35 when adv != NULL).  value_preds[T] is
// overwritten with next_value in the GAE branches, returns[T] with next_value
// otherwise — exactly the reference's side effects.
PPO_API int ppo_compute_returns(const float* rewards, float* value_preds, const float* masks,
                                const float* bad_masks, const float* next_value, float* returns, float* adv,
                                double* partials, int T, int N, double gamma, double gae_lambda, int use_gae,
                                int use_proper_time_limits, void* stream) {
  PPO_REQUIRE(T > 0 && N > 0, "ppo_compute_returns: bad shape T=%d N=%d", T, N);
  PPO_REQUIRE(rewards && value_preds && masks && next_value && returns, "ppo_compute_returns: null pointer");
  PPO_REQUIRE(!use_proper_time_limits || bad_masks, "ppo_compute_returns: bad_masks required");
  PPO_REQUIRE((adv == nullptr) == (partials == nullptr), "ppo_compute_returns: adv and partials go together");
  ProfScope prof("gae", as_stream(stream), (adv ? 20.0 : 16.0) * T * N);
  const float g = (float)gamma;
  const float gl = (float)(gamma * gae_lambda);  // Python double product, then fp32
  hipStream_t st = as_stream(stream);
  const bool F = adv != nullptr;
  if (use_gae) {
    if (use_proper_time_limits)
      return F ? launch_gae<true, true, true>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st)
               : launch_gae<true, true, false>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st);
    return F ? launch_gae<true, false, true>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st)
             : launch_gae<true, false, false>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st);
  }
  if (use_proper_time_limits)
    return F ? launch_gae<false, true, true>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st)
             : launch_gae<false, true, false>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st);
  return F ? launch_gae<false, false, true>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st)
           : launch_gae<false, false, false>(rewards, value_preds, masks, bad_masks, next_value, returns, adv, partials, T, N, g, gl, st);
}

PPO_API int ppo_adv_diff_partials_count(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 2048 ? b : 2048);
}

PPO_API int ppo_adv_diff(const float* returns, const float* value_preds, float* adv, double* partials,
                         long long n, void* stream) {
  PPO_REQUIRE(n > 0, "ppo_adv_diff: n=%lld", n);
  const int blocks = ppo_adv_diff_partials_count(n);
  adv_diff_kernel<<<blocks, 256, 0, as_stream(stream)>>>(returns, value_preds, adv, partials, n);
  PPO_LAUNCH_CHECK("adv_diff_kernel");
  return 0;
}

PPO_API int ppo_adv_finalize(const double* partials, int nparts, double count, double* stats, void* stream) {
  PPO_REQUIRE(nparts > 0, "ppo_adv_finalize: nparts=%d", nparts);
  adv_finalize_kernel<<<1, 256, 0, as_stream(stream)>>>(partials, nparts, count, stats);
  PPO_LAUNCH_CHECK("adv_finalize_kernel");
  return 0;
}

PPO_API int ppo_adv_normalize(float* adv, long long n, const double* stats, void* stream) {
  PPO_REQUIRE(n > 0, "ppo_adv_normalize: n=%lld", n);
  ProfScope prof("adv_norm", as_stream(stream), 8.0 * n);
  long long b = (n + 255) / 256;
  adv_normalize_kernel<<<(unsigned)(b < 4096 ? b : 4096), 256, 0, as_stream(stream)>>>(adv, n, stats);
  PPO_LAUNCH_CHECK("adv_normalize_kernel");
  return 0;
}
