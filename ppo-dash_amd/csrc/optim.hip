// Gradient clipping + Adam on one flat fp32 parameter buffer (K17/K18).
//
// Reference: algo/ppo.py:82-84 —
//   nn.utils.clip_grad_norm_(params, max_grad_norm)   (torch 2.10: total =
//     ‖[‖g_i‖₂]‖₂, coef = min(1, max_norm/(total+1e-6)), g *= coef)
//   optim.Adam(params, lr, eps).step()   (torch 2.10 single-tensor Adam:
//     m.lerp_(g, 1-β1); v = v·β2 + (1-β2)·g²;
//     p -= lr/(1-β1^k) · m / (√v/√(1-β2^k) + eps))
// The norm of the flat buffer equals the norm of the per-tensor norms (up to
// rounding).  `scale` (1/world_size after the RCCL all-reduce) is applied
// before the norm, so every rank clips and steps on the same averaged gradient.
//
// Two launches: fixed-order per-block Σg² partials (double), then one fused
// clip + Adam pass whose blocks each re-reduce the partials in the same order
// (deterministic; no grid-wide sync).  HBM-bound: 4 B·(g + p + m + v) read and
// p, m, v, g written per element.
#include "common.h"

namespace {

constexpr int OPT_THREADS = 256;
constexpr int OPT_MAX_PARTS = 1024;

__global__ __launch_bounds__(OPT_THREADS) void sumsq_kernel(const float* __restrict__ g, long long n, float scale,
                                                           double* __restrict__ partials) {
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < n; i += (long long)gridDim.x * OPT_THREADS) {
    const double x = (double)(g[i] * scale);
    s += x * x;
  }
  __shared__ double r[OPT_THREADS / 64];
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < OPT_THREADS / 64; ++i) t += r[i];
    partials[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(OPT_THREADS) void clip_adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                               float* __restrict__ m, float* __restrict__ v, long long n,
                                                               const double* __restrict__ partials, int nparts,
                                                               float scale, float max_norm, float step_size,
                                                               float bc2_sqrt, float beta1, float beta2, float eps,
                                                               double* __restrict__ norm_out,
                                                               const int* __restrict__ guard_i,
                                                               const double* __restrict__ guard_d,
                                                               int* __restrict__ skipped) {
  // guards (stream-ordered: written by earlier kernels of this minibatch): a timed
  // out persistent GRU launch (*guard_i != 0) or stored actions outside [0, A)
  // (*guard_d > 0) make this step a no-op — parameters, moments and gradient stay
  // bit-unchanged — and count it, so the host can undo its step counter and raise
  const bool skip = (guard_i && *guard_i != 0) || (guard_d && *guard_d > 0.0);
  if (skip) {
    if (skipped && blockIdx.x == 0 && threadIdx.x == 0) *skipped += 1;
    return;
  }
  __shared__ double r[OPT_THREADS];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += OPT_THREADS) s += partials[i];
  r[threadIdx.x] = s;
  __syncthreads();
  for (int o = OPT_THREADS / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
    __syncthreads();
  }
  const float total = (float)sqrt(r[0]);
  float coef = max_norm / (total + 1e-6f);
  coef = coef < 1.0f ? coef : 1.0f;
  if (norm_out && blockIdx.x == 0 && threadIdx.x == 0) norm_out[0] = (double)total;
  const float w = 1.0f - beta1, w2 = 1.0f - beta2;
  for (long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < n; i += (long long)gridDim.x * OPT_THREADS) {
    const float gi = (g[i] * scale) * coef;
    g[i] = gi;  // p.grad holds the clipped gradient afterwards, as in the reference
    float mi = m[i];
    mi = mi + w * (gi - mi);
    float vi = v[i] * beta2;
    vi = vi + w2 * gi * gi;
    const float den = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (-step_size) * (mi / den);
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace

PPO_API int ppo_grad_partials_count(long long n) {
  long long b = (n + OPT_THREADS * 4 - 1) / (OPT_THREADS * 4);
  return (int)(b < 1 ? 1 : (b > OPT_MAX_PARTS ? OPT_MAX_PARTS : b));
}

PPO_API int ppo_grad_sumsq(const float* g, long long n, float scale, double* partials, void* stream) {
  PPO_REQUIRE(n > 0, "ppo_grad_sumsq: n=%lld", n);
  ProfScope prof("grad_sumsq", as_stream(stream), 4.0 * n);
  sumsq_kernel<<<ppo_grad_partials_count(n), OPT_THREADS, 0, as_stream(stream)>>>(g, n, scale, partials);
  PPO_LAUNCH_CHECK("sumsq_kernel");
  return 0;
}

// step: 1-based Adam step count (bias corrections computed here in double, as
// torch does in Python floats).  max_norm <= 0 disables clipping.
PPO_API int ppo_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, long long n,
                          const double* partials, float scale, double max_norm, double lr, double beta1, double beta2,
                          double eps, long long step, double* norm_out, void* stream) {
  return ppo_clip_adam_guarded(params, grads, exp_avg, exp_avg_sq, n, partials, scale, max_norm, lr, beta1, beta2, eps,
                               step, norm_out, nullptr, nullptr, nullptr, stream);
}

PPO_API int ppo_clip_adam_guarded(float* params, float* grads, float* exp_avg, float* exp_avg_sq, long long n,
                                  const double* partials, float scale, double max_norm, double lr, double beta1,
                                  double beta2, double eps, long long step, double* norm_out, const int* guard_i,
                                  const double* guard_d, int* skipped, void* stream) {
  PPO_REQUIRE(n > 0 && step >= 1, "ppo_clip_adam: n=%lld step=%lld", n, step);
  ProfScope prof("clip_adam", as_stream(stream), 28.0 * n);
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float mn = max_norm > 0 ? (float)max_norm : INFINITY;
  long long b = (n + OPT_THREADS - 1) / OPT_THREADS;
  clip_adam_kernel<<<(unsigned)(b < 1024 ? b : 1024), OPT_THREADS, 0, as_stream(stream)>>>(
      params, grads, exp_avg, exp_avg_sq, n, partials, ppo_grad_partials_count(n), scale, mn, step_size, bc2_sqrt,
      (float)beta1, (float)beta2, (float)eps, norm_out, guard_i, guard_d, skipped);
  PPO_LAUNCH_CHECK("clip_adam_kernel");
  return 0;
}
