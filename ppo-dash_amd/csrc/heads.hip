// Actor-critic heads, Categorical distribution and the PPO loss (K13-K15).
//
// Reference:
//   critic_linear / Categorical.linear  model.py:182-199, distributions.py:54-68
//   FixedCategorical sample / log_probs / mode / entropy  distributions.py:17-27
//     (torch Categorical: logits -= logsumexp; probs = softmax(logits);
//      sample = multinomial(probs,1) = argmax(probs / E), E ~ Exp(1);
//      entropy = -Σ logits*probs)
//   Policy.act / evaluate_actions  model.py:54-79
//   PPO clipped surrogate + clipped value loss + entropy  algo/ppo.py:61-81
//
// One wave owns one row at a time.  Lane l holds hidden features
// j = l + 64c (c < HC, H = 64·HC); the head weights for those columns stay in
// registers for all rows the wave processes.  The 1+A head dot products are
// wave-reduced with xor shuffles, so every lane holds value and logits and the
// softmax/sampling/loss arithmetic is computed redundantly (no LDS traffic).
//
// The training kernel is the fused forward + backward of everything above the
// fc layer: loss terms, dL/dlogits and dL/dvalue (analytic, with autograd's
// tie conventions), dL/dfeature masked by the fc ReLU, and per-block partial
// sums of the head weight/bias gradients (deterministic reduce afterwards).
#include "common.h"

namespace {

constexpr int HW = 4;  // waves per block

template <int HC, int AMAX>
struct HeadW {
  float wc[HC];
  float wa[AMAX][HC];
};

template <int HC, int AMAX>
__device__ __forceinline__ void load_head_w(HeadW<HC, AMAX>& w, const float* __restrict__ wc,
                                            const float* __restrict__ wa, int A, int H, int lane) {
#pragma unroll
  for (int c = 0; c < HC; ++c) w.wc[c] = lane + 64 * c < H ? wc[lane + 64 * c] : 0.f;
#pragma unroll
  for (int o = 0; o < AMAX; ++o)
#pragma unroll
    for (int c = 0; c < HC; ++c) w.wa[o][c] = (o < A && lane + 64 * c < H) ? wa[o * H + lane + 64 * c] : 0.f;
}

// value (from fv) and logits (from f) of one row; all lanes end up with the totals
template <int HC, int AMAX>
__device__ __forceinline__ void head_dots(const HeadW<HC, AMAX>& w, const float (&f)[HC], const float (&fv)[HC],
                                          float& value, float (&z)[AMAX], float bc, const float* __restrict__ ba,
                                          int A) {
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < HC; ++c) v += fv[c] * w.wc[c];
  value = wave_sum(v) + bc;
#pragma unroll
  for (int o = 0; o < AMAX; ++o) {
    if (o < A) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < HC; ++c) s += f[c] * w.wa[o][c];
      z[o] = wave_sum(s) + ba[o];
    } else {
      z[o] = -INFINITY;
    }
  }
}

// torch Categorical(logits=z): nl = z - logsumexp(z); p = softmax(nl)
template <int AMAX>
__device__ __forceinline__ void categorical(const float (&z)[AMAX], int A, float (&nl)[AMAX], float (&p)[AMAX]) {
  float mx = z[0];
#pragma unroll
  for (int o = 1; o < AMAX; ++o)
    if (o < A) mx = fmaxf(mx, z[o]);
  float se = 0.f;
#pragma unroll
  for (int o = 0; o < AMAX; ++o)
    if (o < A) se += expf(z[o] - mx);
  const float lse = mx + logf(se);
  float m2 = -INFINITY;
#pragma unroll
  for (int o = 0; o < AMAX; ++o) {
    nl[o] = o < A ? z[o] - lse : -INFINITY;
    if (o < A) m2 = fmaxf(m2, nl[o]);
  }
  float s2 = 0.f;
#pragma unroll
  for (int o = 0; o < AMAX; ++o) {
    p[o] = o < A ? expf(nl[o] - m2) : 0.f;
    s2 += p[o];
  }
#pragma unroll
  for (int o = 0; o < AMAX; ++o) p[o] = p[o] / s2;
}

__device__ __forceinline__ float exp_noise(uint64_t seed, uint64_t counter, long long row, int o, int A) {
  const uint64_t h = mix64(seed ^ mix64(counter * 0x2545F4914F6CDD1Dull + (uint64_t)(row * A + o)));
  return -logf(u01_open0(h));
}

// act / evaluate: value, action (sample | mode | given), log_prob, entropy
// FAST: A == AMAX, H == 64·HC, no separate critic features (compile-time bounds)
template <int HC, int AMAX, bool FAST>
__global__ __launch_bounds__(64 * HW) void heads_act_kernel(
    const float* __restrict__ feat, const float* __restrict__ feat_v_, int N, int H_, const float* __restrict__ wc,
    const float* __restrict__ bc, const float* __restrict__ wa, const float* __restrict__ ba, int A_,
    const float* __restrict__ noise,
    unsigned long long seed, unsigned long long counter, int deterministic, const int64_t* __restrict__ given,
    float* __restrict__ value_out, int64_t* __restrict__ action_out, float* __restrict__ logp_out,
    float* __restrict__ ent_out, int rows_per_wave) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int H = FAST ? 64 * HC : H_, A = FAST ? AMAX : A_;
  const float* const feat_v = FAST ? nullptr : feat_v_;
  HeadW<HC, AMAX> w;
  load_head_w(w, wc, wa, A, H, lane);
  const float b0 = bc[0];
  const long long r0 = ((long long)blockIdx.x * HW + wave) * rows_per_wave;
  for (int rr = 0; rr < rows_per_wave; ++rr) {
    const long long row = r0 + rr;
    if (row >= N) break;
    float f[HC], fv[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      const bool in = lane + 64 * c < H;
      f[c] = in ? feat[row * H + lane + 64 * c] : 0.f;
      fv[c] = feat_v ? (in ? feat_v[row * H + lane + 64 * c] : 0.f) : f[c];
    }
    float value, z[AMAX], nl[AMAX], p[AMAX];
    head_dots(w, f, fv, value, z, b0, ba, A);
    categorical(z, A, nl, p);
    int act;
    if (given) {
      act = (int)given[row];
    } else {
      act = 0;
      float best = -INFINITY;
#pragma unroll
      for (int o = 0; o < AMAX; ++o) {
        if (o < A) {
          const float sc = deterministic ? p[o] : p[o] / (noise ? noise[row * A + o] : exp_noise(seed, counter, row, o, A));
          if (sc > best) { best = sc; act = o; }
        }
      }
    }
    // an action index outside [0, A) has no log-prob: the reference's gather
    // raises there (distributions.py:22); NaN marks the row here
    float lp = (unsigned)act < (unsigned)A ? 0.f : __int_as_float(0x7fc00000), ent = 0.f;
#pragma unroll
    for (int o = 0; o < AMAX; ++o) {
      if (o == act && o < A) lp = nl[o];
      if (o < A) ent -= nl[o] * p[o];
    }
    if (lane == 0) {
      if (value_out) value_out[row] = value;
      if (action_out) action_out[row] = act;
      if (logp_out) logp_out[row] = lp;
      if (ent_out) ent_out[row] = ent;
    }
  }
}

// d(pre-activation) from d(output) for the activation that produced y
__device__ __forceinline__ float act_grad(float d, float y, int act) {
  if (act == 1) return y > 0.f ? d : 0.f;     // ReLU (threshold_backward)
  if (act == 2) return d * (1.0f - y * y);    // tanh
  return d;
}

struct TrainArgs {
  const float* feat;  // [B][H] policy features (CNNBase: post-ReLU fc; MLPBase: actor tanh output)
  const float* feat_v;  // [B][H] critic features (MLPBase) or NULL (= feat)
  int B, H, A;
  const float *wc, *bc, *wa, *ba;
  const int64_t* idx;      // storage row of each sample (nullable: row0 + b)
  long long row0;
  const int64_t* actions;  // storage planes, indexed by storage row
  const float *old_logp, *adv, *vpred, *ret;
  float clip, value_coef, entropy_coef, inv_b;
  int use_clipped_value_loss;
  int feat_act;            // activation producing the features: 0 none (GRU), 1 ReLU, 2 tanh
  float* dfeat;            // [B][H] dL/d(feature pre-activation) (both heads when dfeat_v is NULL)
  float* dfeat_v;          // [B][H] critic-branch gradient (MLPBase) or NULL
  float* part_w;           // [blocks][1+A][H]
  float* part_b;           // [blocks][1+A]
  float* part_loss;        // [blocks][4]: Σ max(l1,l2), Σ min(s1,s2), Σ H, # actions outside [0, A)
  int rows_per_wave;
};

// FAST: A == AMAX, H == 64·HC, no separate critic features / gradient (CNNBase
// and the GRU policy): every per-lane and per-action bound is a compile-time
// constant, which removes the uniform branches around each unrolled operation
// (the generic instantiation runs ~2,500 instructions per row).
template <int HC, int AMAX, bool FAST>
__global__ __launch_bounds__(64 * HW) void heads_train_kernel(const TrainArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int H = FAST ? 64 * HC : a.H, A = FAST ? AMAX : a.A;
  const float* const feat_v = FAST ? nullptr : a.feat_v;
  float* const dfeat_v = FAST ? nullptr : a.dfeat_v;
  HeadW<HC, AMAX> w;
  load_head_w(w, a.wc, a.wa, A, H, lane);
  const float b0 = a.bc[0];
  float gwc[HC], gwa[AMAX][HC], gbc = 0.f, gba[AMAX];
#pragma unroll
  for (int c = 0; c < HC; ++c) gwc[c] = 0.f;
#pragma unroll
  for (int o = 0; o < AMAX; ++o) {
    gba[o] = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c) gwa[o][c] = 0.f;
  }
  float s_vl = 0.f, s_al = 0.f, s_ent = 0.f, s_bad = 0.f;
  const float clip = a.clip;
  const long long r0 = ((long long)blockIdx.x * HW + wave) * a.rows_per_wave;
  // The per-row storage scalars (the minibatch gather idx -> action, advantage,
  // old log-prob, value, return) of all of this wave's rows are fetched up
  // front, lane j holding row r0 + j (rows_per_wave <= 64), and broadcast with
  // readlane per row; each row's features are loaded one row ahead.  Without
  // this the wave waited on two dependent loads per row (latency-bound).
  int q_act = 0;
  float q_adv = 0.f, q_olp = 0.f, q_vo = 0.f, q_ret = 0.f;
  if (lane < a.rows_per_wave && r0 + lane < a.B) {
    const long long sr = a.idx ? (long long)a.idx[r0 + lane] : a.row0 + r0 + lane;
    q_act = (int)a.actions[sr];
    q_adv = a.adv[sr];
    q_olp = a.old_logp[sr];
    q_vo = a.vpred[sr];
    q_ret = a.ret[sr];
  }
  auto bcast = [](float x, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j));
  };
  float fn[HC], fvn[HC];
  auto load_row = [&](long long row) {
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      const bool in = row < a.B && lane + 64 * c < H;
      fn[c] = in ? a.feat[row * H + lane + 64 * c] : 0.f;
      fvn[c] = feat_v ? (in ? feat_v[row * H + lane + 64 * c] : 0.f) : fn[c];
    }
  };
  load_row(r0);
  for (int rr = 0; rr < a.rows_per_wave; ++rr) {
    const long long row = r0 + rr;
    if (row >= a.B) break;
    float f[HC], fv[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      f[c] = fn[c];
      fv[c] = fvn[c];
    }
    if (rr + 1 < a.rows_per_wave) load_row(row + 1);
    float value, z[AMAX], nl[AMAX], p[AMAX];
    head_dots(w, f, fv, value, z, b0, a.ba, A);
    categorical(z, A, nl, p);
    const int act = __builtin_amdgcn_readlane(q_act, rr);
    s_bad += (unsigned)act < (unsigned)A ? 0.f : 1.f;   // counted; PPO.update raises (gather's IndexError)
    float lp = 0.f, ent = 0.f;
#pragma unroll
    for (int o = 0; o < AMAX; ++o) {
      if (o == act) lp = nl[o];
      if (o < A) ent -= nl[o] * p[o];
    }
    // action loss (ppo.py:61-66)
    const float adv = bcast(q_adv, rr);
    const float ratio = expf(lp - bcast(q_olp, rr));
    const float surr1 = ratio * adv;
    const float rc = fminf(fmaxf(ratio, 1.0f - clip), 1.0f + clip);
    const float surr2 = rc * adv;
    const float w1 = surr1 < surr2 ? 1.f : (surr1 == surr2 ? 0.5f : 0.f);
    const float inr = (ratio >= 1.0f - clip && ratio <= 1.0f + clip) ? 1.f : 0.f;
    const float g_logp = -a.inv_b * (w1 * adv + (1.f - w1) * adv * inr) * ratio;
    // value loss (ppo.py:68-77)
    const float vo = bcast(q_vo, rr), R = bcast(q_ret, rr);
    float g_v, vl_row;
    if (a.use_clipped_value_loss) {
      const float dv = value - vo;
      const float vpc = vo + fminf(fmaxf(dv, -clip), clip);
      const float l1 = (value - R) * (value - R);
      const float l2 = (vpc - R) * (vpc - R);
      vl_row = fmaxf(l1, l2);
      const float u1 = l1 > l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
      const float vin = (dv >= -clip && dv <= clip) ? 1.f : 0.f;
      g_v = a.value_coef * 0.5f * a.inv_b * (u1 * 2.f * (value - R) + (1.f - u1) * 2.f * (vpc - R) * vin);
    } else {
      vl_row = (R - value) * (R - value);
      g_v = a.value_coef * a.inv_b * (value - R);
    }
    s_vl += vl_row;
    s_al += fminf(surr1, surr2);
    s_ent += ent;
    // dL/dlogits = g_logp (onehot - p) + (c_e/B) p (nl + H)
    float gz[AMAX];
    const float ce = a.entropy_coef * a.inv_b;
#pragma unroll
    for (int o = 0; o < AMAX; ++o)
      gz[o] = o < A ? g_logp * ((o == act ? 1.f : 0.f) - p[o]) + ce * p[o] * (nl[o] + ent) : 0.f;
    // dL/dh for this lane's columns, masked by the fc ReLU; head grads
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      const float dv = g_v * w.wc[c];
      float d = dfeat_v ? 0.f : dv;
#pragma unroll
      for (int o = 0; o < AMAX; ++o) d += gz[o] * w.wa[o][c];
      if (lane + 64 * c < H) {
        const size_t q = (size_t)row * H + lane + 64 * c;
        a.dfeat[q] = act_grad(d, f[c], a.feat_act);
        if (dfeat_v) dfeat_v[q] = act_grad(dv, fv[c], a.feat_act);
      }
      gwc[c] += g_v * fv[c];
#pragma unroll
      for (int o = 0; o < AMAX; ++o) gwa[o][c] += gz[o] * f[c];
    }
    gbc += g_v;
#pragma unroll
    for (int o = 0; o < AMAX; ++o) gba[o] += gz[o];
  }
  // block reduction of the head-gradient partials across the HW waves
  __shared__ float red[HW][64 * HC];
  __shared__ float redb[HW][AMAX + 5];
  const int NO = 1 + A;
  for (int o = 0; o < NO; ++o) {
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      float v = gwc[c];
#pragma unroll
      for (int q = 0; q < AMAX; ++q)
        if (o == q + 1) v = gwa[q][c];
      red[wave][lane + 64 * c] = v;
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int c = 0; c < HC; ++c) {
        const int j = lane + 64 * c;
        float s = red[0][j];
        for (int q = 1; q < HW; ++q) s += red[q][j];
        if (j < H) a.part_w[((size_t)blockIdx.x * NO + o) * H + j] = s;
      }
    }
    __syncthreads();
  }
  if (lane == 0) {
    redb[wave][0] = gbc;
#pragma unroll
    for (int o = 0; o < AMAX; ++o) redb[wave][1 + o] = gba[o];
    redb[wave][AMAX + 1] = s_vl;
    redb[wave][AMAX + 2] = s_al;
    redb[wave][AMAX + 3] = s_ent;
    redb[wave][AMAX + 4] = s_bad;
  }
  __syncthreads();
  if (threadIdx.x < NO) {
    float s = 0.f;
    for (int q = 0; q < HW; ++q) s += redb[q][threadIdx.x];
    a.part_b[(size_t)blockIdx.x * NO + threadIdx.x] = s;
  }
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int q = 0; q < HW; ++q) s += redb[q][AMAX + 1 + threadIdx.x];
    a.part_loss[(size_t)blockIdx.x * 4 + threadIdx.x] = s;
  }
}

// heads_train_kernel for CNNBase / the GRU policy at H = 512, A = 8 (TrainArgs'
// FAST case) with the head weights in LDS instead of registers: a lane holds the
// columns 4·lane + q + 256·c2 (q < 4, c2 < 2: float4 loads and stores of the
// features and their gradient) and reads the 9 weight rows of those columns as
// 18 ds_read_b128 per row pass.  The register version held 72 weight VGPRs next
// to the 72 gradient accumulators (256 VGPRs: one wave per SIMD, every row's
// dependent chain — 9 wave reductions, the softmax, the loss — exposed); this one
// fits two waves per SIMD.  Same arithmetic per element, same partial layout.
__global__ __launch_bounds__(64 * HW) void heads_train_lds_kernel(const TrainArgs a) {
  constexpr int A = 8, H = 512;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ f32x4 Wl[9][128];   // row 0: critic, rows 1..8: actor logits (the flat parameter
  for (int i = threadIdx.x; i < 9 * H; i += 64 * HW) {   // buffer places wa at an odd offset: scalar loads)
    const int o = i / H, k = i - H * o;
    reinterpret_cast<float*>(&Wl[o][0])[k] = o == 0 ? a.wc[k] : a.wa[(o - 1) * H + k];
  }
  const float b0 = a.bc[0];
  float ba[A];
#pragma unroll
  for (int o = 0; o < A; ++o) ba[o] = a.ba[o];
  __syncthreads();
  f32x4 gw[9][2];   // Σ_rows g_o · f (o = 0: critic), this lane's columns
#pragma unroll
  for (int o = 0; o < 9; ++o) gw[o][0] = gw[o][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gbc = 0.f, gba[A];
#pragma unroll
  for (int o = 0; o < A; ++o) gba[o] = 0.f;
  float s_vl = 0.f, s_al = 0.f, s_ent = 0.f, s_bad = 0.f;
  const float clip = a.clip;
  const long long r0 = ((long long)blockIdx.x * HW + wave) * a.rows_per_wave;
  int q_act = 0;
  float q_adv = 0.f, q_olp = 0.f, q_vo = 0.f, q_ret = 0.f;
  if (lane < a.rows_per_wave && r0 + lane < a.B) {
    const long long sr = a.idx ? (long long)a.idx[r0 + lane] : a.row0 + r0 + lane;
    q_act = (int)a.actions[sr];
    q_adv = a.adv[sr];
    q_olp = a.old_logp[sr];
    q_vo = a.vpred[sr];
    q_ret = a.ret[sr];
  }
  auto bcast = [](float x, int j) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j)); };
  f32x4 fn[2];
  auto load_row = [&](long long row) {
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
      fn[c2] = row < a.B ? reinterpret_cast<const f32x4*>(a.feat + row * H)[lane + 64 * c2] : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  load_row(r0);
  for (int rr = 0; rr < a.rows_per_wave; ++rr) {
    const long long row = r0 + rr;
    if (row >= a.B) break;
    const f32x4 f[2] = {fn[0], fn[1]};
    if (rr + 1 < a.rows_per_wave) load_row(row + 1);
    float dots[9];
#pragma unroll
    for (int o = 0; o < 9; ++o) {
      float t = 0.f;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const f32x4 w = Wl[o][lane + 64 * c2];
#pragma unroll
        for (int q = 0; q < 4; ++q) t += f[c2][q] * w[q];
      }
      dots[o] = wave_sum(t);
    }
    const float value = dots[0] + b0;
    float z[A], nl[A], p[A];
#pragma unroll
    for (int o = 0; o < A; ++o) z[o] = dots[1 + o] + ba[o];
    categorical(z, A, nl, p);
    const int act = __builtin_amdgcn_readlane(q_act, rr);
    s_bad += (unsigned)act < (unsigned)A ? 0.f : 1.f;
    float lp = 0.f, ent = 0.f;
#pragma unroll
    for (int o = 0; o < A; ++o) {
      if (o == act) lp = nl[o];
      ent -= nl[o] * p[o];
    }
    // action loss (ppo.py:61-66)
    const float adv = bcast(q_adv, rr);
    const float ratio = expf(lp - bcast(q_olp, rr));
    const float surr1 = ratio * adv;
    const float rc = fminf(fmaxf(ratio, 1.0f - clip), 1.0f + clip);
    const float surr2 = rc * adv;
    const float w1 = surr1 < surr2 ? 1.f : (surr1 == surr2 ? 0.5f : 0.f);
    const float inr = (ratio >= 1.0f - clip && ratio <= 1.0f + clip) ? 1.f : 0.f;
    const float g_logp = -a.inv_b * (w1 * adv + (1.f - w1) * adv * inr) * ratio;
    // value loss (ppo.py:68-77)
    const float vo = bcast(q_vo, rr), R = bcast(q_ret, rr);
    float g_v, vl_row;
    if (a.use_clipped_value_loss) {
      const float dv = value - vo;
      const float vpc = vo + fminf(fmaxf(dv, -clip), clip);
      const float l1 = (value - R) * (value - R);
      const float l2 = (vpc - R) * (vpc - R);
      vl_row = fmaxf(l1, l2);
      const float u1 = l1 > l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
      const float vin = (dv >= -clip && dv <= clip) ? 1.f : 0.f;
      g_v = a.value_coef * 0.5f * a.inv_b * (u1 * 2.f * (value - R) + (1.f - u1) * 2.f * (vpc - R) * vin);
    } else {
      vl_row = (R - value) * (R - value);
      g_v = a.value_coef * a.inv_b * (value - R);
    }
    s_vl += vl_row;
    s_al += fminf(surr1, surr2);
    s_ent += ent;
    float g[9];   // g[0] = dL/dvalue, g[1 + o] = dL/dlogit o
    g[0] = g_v;
    const float ce = a.entropy_coef * a.inv_b;
#pragma unroll
    for (int o = 0; o < A; ++o) g[1 + o] = g_logp * ((o == act ? 1.f : 0.f) - p[o]) + ce * p[o] * (nl[o] + ent);
    // dL/dfeature of this lane's columns (masked by the activation), head gradients
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
      f32x4 d = Wl[0][lane + 64 * c2] * g[0];
#pragma unroll
      for (int o = 1; o < 9; ++o) {
        const f32x4 w = Wl[o][lane + 64 * c2];
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] += g[o] * w[q];
      }
      f32x4 y;
#pragma unroll
      for (int q = 0; q < 4; ++q) y[q] = act_grad(d[q], f[c2][q], a.feat_act);
      reinterpret_cast<f32x4*>(a.dfeat + row * H)[lane + 64 * c2] = y;
#pragma unroll
      for (int o = 0; o < 9; ++o)
#pragma unroll
        for (int q = 0; q < 4; ++q) gw[o][c2][q] += g[o] * f[c2][q];
    }
    gbc += g_v;
#pragma unroll
    for (int o = 0; o < A; ++o) gba[o] += g[1 + o];
  }
  // block reduction of the head-gradient partials across the HW waves (fixed order)
  __shared__ f32x4 red[HW][128];
  __shared__ float redb[HW][A + 5];
  for (int o = 0; o < 9; ++o) {
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) red[wave][lane + 64 * c2] = gw[o][c2];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        f32x4 t = red[0][lane + 64 * c2];
        for (int q = 1; q < HW; ++q) t += red[q][lane + 64 * c2];
        reinterpret_cast<f32x4*>(a.part_w + ((size_t)blockIdx.x * 9 + o) * H)[lane + 64 * c2] = t;
      }
    }
    __syncthreads();
  }
  if (lane == 0) {
    redb[wave][0] = gbc;
#pragma unroll
    for (int o = 0; o < A; ++o) redb[wave][1 + o] = gba[o];
    redb[wave][A + 1] = s_vl;
    redb[wave][A + 2] = s_al;
    redb[wave][A + 3] = s_ent;
    redb[wave][A + 4] = s_bad;
  }
  __syncthreads();
  if (threadIdx.x < 9) {
    float t = 0.f;
    for (int q = 0; q < HW; ++q) t += redb[q][threadIdx.x];
    a.part_b[(size_t)blockIdx.x * 9 + threadIdx.x] = t;
  }
  if (threadIdx.x < 4) {
    float t = 0.f;
    for (int q = 0; q < HW; ++q) t += redb[q][A + 1 + threadIdx.x];
    a.part_loss[(size_t)blockIdx.x * 4 + threadIdx.x] = t;
  }
}

// loss partials -> acc[0..3] += {0.5·Σvl/B, -Σal/B, Σent/B, # bad actions} (double, fixed order)
__global__ __launch_bounds__(256) void loss_reduce_kernel(const float* __restrict__ part_loss, int nblk,
                                                          double* __restrict__ loss_acc, double inv_b) {
  __shared__ double r[4][256];
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nblk; b += 256)
    for (int q = 0; q < 4; ++q) acc[q] += (double)part_loss[(size_t)b * 4 + q];
  for (int q = 0; q < 4; ++q) r[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int q = 0; q < 4; ++q) r[q][threadIdx.x] += r[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    loss_acc[0] += 0.5 * r[0][0] * inv_b;
    loss_acc[1] += -r[1][0] * inv_b;
    loss_acc[2] += r[2][0] * inv_b;
    loss_acc[3] += r[3][0];
  }
}

__global__ __launch_bounds__(256) void mean_kernel(const float* __restrict__ x, long long n, float* __restrict__ out) {
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) s += (double)x[i];
  __shared__ double r[256];
  r[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(r[0] / (double)n);
}

// 64-column chunks per lane, rounded up to an instantiated count (1, 2, 4, 8)
static inline int hc_of(int H) {
  const int c = (H + 63) / 64;
  return c <= 1 ? 1 : c <= 2 ? 2 : c <= 4 ? 4 : 8;
}

template <int HC, int AMAX>
int launch_act(const float* feat, const float* feat_v, int N, int H, const float* wc, const float* bc, const float* wa,
               const float* ba,
               int A, const float* noise, unsigned long long seed, unsigned long long counter, int det,
               const int64_t* given, float* v, int64_t* act, float* lp, float* ent, hipStream_t st) {
  // ~4096 waves in flight (4 per SIMD at this kernel's 122-137 VGPRs): a rollout batch of
  // 4,096 rows takes one row per wave, so no wave runs two rows' dependent chains back to back
  const int rpw = (int)std::min<long long>(8, std::max<long long>(1, ceil_div(N, 4096)));
  const unsigned blocks = ceil_div(N, HW * rpw);
  if (A == AMAX && H == 64 * HC && !feat_v)
    heads_act_kernel<HC, AMAX, true><<<blocks, 64 * HW, 0, st>>>(feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter,
                                                        det,
                                                        given, v, act, lp, ent, rpw);
  else
    heads_act_kernel<HC, AMAX, false><<<blocks, 64 * HW, 0, st>>>(feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter,
                                                        det,
                                                        given, v, act, lp, ent, rpw);
  PPO_LAUNCH_CHECK("heads_act_kernel");
  return 0;
}

template <int AMAX>
int dispatch_act(int HC, const float* feat, const float* feat_v, int N, int H, const float* wc, const float* bc,
                 const float* wa,
                 const float* ba, int A, const float* noise, unsigned long long seed, unsigned long long counter,
                 int det, const int64_t* given, float* v, int64_t* act, float* lp, float* ent, hipStream_t st) {
  switch (HC) {
    case 1: return launch_act<1, AMAX>(feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter, det, given, v, act, lp, ent, st);
    case 2: return launch_act<2, AMAX>(feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter, det, given, v, act, lp, ent, st);
    case 4: return launch_act<4, AMAX>(feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter, det, given, v, act, lp, ent, st);
    case 8: return launch_act<8, AMAX>(feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter, det, given, v, act, lp, ent, st);
  }
  ppo_set_error("heads: hidden size %d not supported (<= 512)", H);
  return PPO_EARG;
}

static int g_heads_lds = 1;   // ppo_tune_set("heads_lds", 0): the register-weight kernel (A/B)

template <int HC, int AMAX>
int launch_train(const TrainArgs& a, int blocks, hipStream_t st) {
  if (g_heads_lds && HC == 8 && AMAX == 8 && a.A == 8 && a.H == 512 && !a.feat_v && !a.dfeat_v &&
      ((uintptr_t)a.feat & 15) == 0 && ((uintptr_t)a.dfeat & 15) == 0 && ((uintptr_t)a.part_w & 15) == 0) {
    heads_train_lds_kernel<<<blocks, 64 * HW, 0, st>>>(a);
    PPO_LAUNCH_CHECK("heads_train_lds_kernel");
    return 0;
  }
  if (a.A == AMAX && a.H == 64 * HC && !a.feat_v && !a.dfeat_v)
    heads_train_kernel<HC, AMAX, true><<<blocks, 64 * HW, 0, st>>>(a);
  else
    heads_train_kernel<HC, AMAX, false><<<blocks, 64 * HW, 0, st>>>(a);
  PPO_LAUNCH_CHECK("heads_train_kernel");
  return 0;
}

template <int AMAX>
int dispatch_train(int HC, const TrainArgs& a, int blocks, hipStream_t st) {
  switch (HC) {
    case 1: return launch_train<1, AMAX>(a, blocks, st);
    case 2: return launch_train<2, AMAX>(a, blocks, st);
    case 4: return launch_train<4, AMAX>(a, blocks, st);
    case 8: return launch_train<8, AMAX>(a, blocks, st);
  }
  ppo_set_error("heads: hidden size %d not supported (<= 512)", a.H);
  return PPO_EARG;
}

}  // namespace

// Policy.act / evaluate_actions heads (model.py:54-79):
//   noise   != NULL: sample = argmax(probs / noise) (host-replay parity mode)
//   noise   == NULL: Exp(1) noise from the counter RNG (seed, counter, row)
//   given   != NULL: log_prob/entropy of the given actions (evaluate_actions)
//   deterministic: mode = argmax(probs)
PPO_API int ppo_heads_act(const float* feat, const float* feat_v, int N, int H, const float* wc, const float* bc,
                          const float* wa,
                          const float* ba, int A, const float* noise, unsigned long long seed,
                          unsigned long long counter, int deterministic, const int64_t* given, float* value,
                          int64_t* action, float* logp, float* entropy, void* stream) {
  PPO_REQUIRE(N >= 0 && A >= 1 && A <= 16, "ppo_heads_act: N=%d A=%d (1..16 actions)", N, A);
  PPO_REQUIRE(H > 0 && H <= 512, "ppo_heads_act: hidden size %d (1..512)", H);
  ProfScope prof("heads_act", as_stream(stream), (double)N * (4.0 * H * (feat_v ? 2 : 1) + 16.0));
  if (N == 0) return 0;
  hipStream_t st = as_stream(stream);
  const int HC = hc_of(H);
  if (A <= 8)
    return dispatch_act<8>(HC, feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter, deterministic, given, value,
                           action, logp, entropy, st);
  return dispatch_act<16>(HC, feat, feat_v, N, H, wc, bc, wa, ba, A, noise, seed, counter, deterministic, given, value,
                          action, logp, entropy, st);
}

int heads_lds_knob(int set, int value) {   // gemm.hip's ppo_tune_set / _get ("heads_lds")
  if (set) g_heads_lds = value;
  return g_heads_lds;
}

PPO_API int ppo_heads_train_blocks(int B) {
  const int rpw = 32;
  return (int)ceil_div(B, HW * rpw);
}

PPO_API int ppo_heads_train(const float* feat, const float* feat_v, int B, int H, const float* wc, const float* bc,
                            const float* wa,
                            const float* ba, int A, const int64_t* idx, long long row0, const int64_t* actions,
                            const float* old_logp, const float* adv, const float* vpred, const float* ret, float clip,
                            float value_coef, float entropy_coef, float inv_b, int use_clipped_value_loss,
                            int feat_act, float* dfeat, float* dfeat_v, float* part_w, float* part_b,
                            float* part_loss, void* stream) {
  PPO_REQUIRE(B > 0 && A >= 1 && A <= 16, "ppo_heads_train: B=%d A=%d", B, A);
  PPO_REQUIRE(H > 0 && H <= 512, "ppo_heads_train: hidden size %d (1..512)", H);
  ProfScope prof("heads_train", as_stream(stream),
                 (double)B * (8.0 * H * (feat_v ? 2 : 1) + (idx ? 8.0 : 0.0) + 32.0));
  TrainArgs a;
  a.feat = feat; a.feat_v = feat_v; a.B = B; a.H = H; a.A = A; a.wc = wc; a.bc = bc; a.wa = wa; a.ba = ba;
  a.idx = idx; a.row0 = row0; a.actions = actions; a.old_logp = old_logp; a.adv = adv; a.vpred = vpred; a.ret = ret;
  a.clip = clip; a.value_coef = value_coef; a.entropy_coef = entropy_coef; a.inv_b = inv_b;
  a.use_clipped_value_loss = use_clipped_value_loss;
  a.feat_act = feat_act;
  a.dfeat_v = dfeat_v;
  a.dfeat = dfeat; a.part_w = part_w; a.part_b = part_b; a.part_loss = part_loss;
  a.rows_per_wave = 32;
  const int blocks = ppo_heads_train_blocks(B);
  hipStream_t st = as_stream(stream);
  if (A <= 8) return dispatch_train<8>(hc_of(H), a, blocks, st);
  return dispatch_train<16>(hc_of(H), a, blocks, st);
}

// Σ over the heads_train blocks (fixed order) -> head gradients; losses -> loss_acc
PPO_API int ppo_heads_reduce(const float* part_w, const float* part_b, const float* part_loss, int nblk, int H, int A,
                             float* g_wc, float* g_bc, float* g_wa, float* g_ba, double* loss_acc, double inv_b,
                             float scale, int use_clipped_value_loss, void* stream) {
  (void)use_clipped_value_loss;  // both value losses are 0.5·mean(·)
  ProfScope prof("heads_reduce", as_stream(stream), 4.0 * nblk * (1.0 + A) * (H + 1));
  const long long NO = 1 + A;
  int rc;
  if ((rc = ppo_colsum(part_w, NO * H, nblk, H, g_wc, scale, 0, stream))) return rc;
  if ((rc = ppo_colsum(part_w + H, NO * H, nblk, (long long)A * H, g_wa, scale, 0, stream))) return rc;
  if ((rc = ppo_colsum(part_b, NO, nblk, 1, g_bc, scale, 0, stream))) return rc;
  if ((rc = ppo_colsum(part_b + 1, NO, nblk, A, g_ba, scale, 0, stream))) return rc;
  if (loss_acc) {
    loss_reduce_kernel<<<1, 256, 0, as_stream(stream)>>>(part_loss, nblk, loss_acc, inv_b);
    PPO_LAUNCH_CHECK("loss_reduce_kernel");
  }
  return 0;
}

PPO_API int ppo_mean_f32(const float* x, long long n, float* out, void* stream) {
  PPO_REQUIRE(n > 0, "ppo_mean_f32: n=%lld", n);
  mean_kernel<<<1, 256, 0, as_stream(stream)>>>(x, n, out);
  PPO_LAUNCH_CHECK("mean_kernel");
  return 0;
}
