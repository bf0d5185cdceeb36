/*
 * ORACLE — test infrastructure only.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * or the timed CPU baseline; the product path never links or calls it.
 *
 * Scalar C restatement of RolloutStorage.compute_returns
 * (ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/storage.py:82-121,
 * identical in ppo-dash-study/001_baseline/ppo/storage.py:82-121), in the
 * reference's fp32 operation order.  Pinned bit-exactly by tests/golden/gae.npz.
 *
 * Operation order, as torch evaluates the Python expressions on fp32 tensors
 * with Python-float scalars (the scalar is rounded to fp32 first):
 *   delta = ((r_t + (fl(g) * v_{t+1}) * m_{t+1}) - v_t)          :93-95 / :111-113
 *   gae   = delta + ((fl(g*lam) * m_{t+1}) * gae)                  :96-97 / :114-115
 *           (g*lam is a Python double product, rounded once)
 *   gae   = gae * bm_{t+1}                        (time limits)   :98
 *   ret_t = gae + v_t                                              :99 / :116
 * non-GAE:
 *   ret_t = ((ret_{t+1} * fl(g)) * m_{t+1}) + r_t                  :120-121
 *   time limits: ((ret_{t+1}*g)*m + r)*bm + (1 - bm)*v_t           :103-105
 * The GAE branches overwrite value_preds[T] with next_value (:90, :108) and leave
 * returns[T] untouched; the non-GAE branches set returns[T] = next_value.
 *
 * Build with -ffp-contract=off: an FMA would change the rounding.
 * Layout: all arrays [T(+1)][N] row-major (time-major, env-minor), as the
 * reference's [T(+1), N, 1] tensors.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

void oracle_compute_returns(const float *rewards,   /* [T][N]   */
                            float *value_preds,     /* [T+1][N] (row T overwritten if use_gae) */
                            const float *masks,     /* [T+1][N] */
                            const float *bad_masks, /* [T+1][N] */
                            const float *next_value,/* [N]      */
                            float *returns,         /* [T+1][N] */
                            int T, int N, double gamma, double gae_lambda,
                            int use_gae, int use_proper_time_limits)
{
    const float g = (float)gamma;
    const float gl = (float)(gamma * gae_lambda);
    if (use_gae) {
        for (int n = 0; n < N; ++n) value_preds[(size_t)T * N + n] = next_value[n];
        for (int n = 0; n < N; ++n) {
            float gae = 0.0f;
            for (int t = T - 1; t >= 0; --t) {
                const size_t i = (size_t)t * N + n, i1 = (size_t)(t + 1) * N + n;
                float a = g * value_preds[i1];
                a = a * masks[i1];
                float delta = rewards[i] + a;
                delta = delta - value_preds[i];
                float b = gl * masks[i1];
                b = b * gae;
                gae = delta + b;
                if (use_proper_time_limits) gae = gae * bad_masks[i1];
                returns[i] = gae + value_preds[i];
            }
        }
    } else {
        for (int n = 0; n < N; ++n) returns[(size_t)T * N + n] = next_value[n];
        for (int n = 0; n < N; ++n) {
            for (int t = T - 1; t >= 0; --t) {
                const size_t i = (size_t)t * N + n, i1 = (size_t)(t + 1) * N + n;
                float x = returns[i1] * g;
                x = x * masks[i1];
                x = x + rewards[i];
                if (use_proper_time_limits) {
                    x = x * bad_masks[i1];
                    float keep = 1.0f - bad_masks[i1];
                    keep = keep * value_preds[i];
                    x = x + keep;
                }
                returns[i] = x;
            }
        }
    }
}

/* Advantage statistics for ppo.py:35-37: adv = returns[:-1] - value_preds[:-1],
 * mean and unbiased std over all T*N elements.  The differences are fp32 (as in
 * torch); the moments are accumulated in double.  out[0]=mean, out[1]=std. */
void oracle_adv_stats(const float *returns, const float *value_preds, int T, int N, double *out)
{
    const size_t n = (size_t)T * N;
    double s = 0.0;
    for (size_t i = 0; i < n; ++i) s += (double)(returns[i] - value_preds[i]);
    const double mean = s / (double)n;
    double m2 = 0.0;
    for (size_t i = 0; i < n; ++i) {
        const double d = (double)(returns[i] - value_preds[i]) - mean;
        m2 += d * d;
    }
    out[0] = mean;
    out[1] = n > 1 ? sqrt(m2 / (double)(n - 1)) : NAN;
}

/* The device decode of u8 observations (common.h decode_u8): q = u*(1/255),
 * one residual FMA correction.  Exposed so the CPU tests can check it against
 * IEEE u/255.0f for all 256 codes. */
float oracle_decode_u8_fma(unsigned u)
{
    const float r = 1.0f / 255.0f;
    const float x = (float)u;
    const float q = x * r;
    const float res = fmaf(-q, 255.0f, x);
    return fmaf(res, r, q);
}
