// Rollout storage kernels (K1/K2/K5/K6) and the synthetic on-GPU environment.
//
// Reference: RolloutStorage (ppo-dash-training/pytorch-a2c-ppo-acktr-gail/
// a2c_ppo_acktr/storage.py): insert :60-73, after_update :75-80,
// feed_forward_generator gather :138-160, recurrent_generator :162-223.
//
// HBM layout (structure of arrays, one plane per field):
//   obs        u8  [T+1][N][C][84][84]   (28,224 B per env-step row, 16-B aligned)
//   rewards    f32 [T][N]   value_preds/returns/masks/bad_masks f32 [T+1][N]
//   actions    i64 [T][N]   action_log_probs f32 [T][N]
// Every kernel here is a byte mover: HBM-bound, 16-B vector accesses.
#include <stdarg.h>
#include <string.h>

#include "common.h"

static thread_local char g_err[512] = "";

void ppo_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

PPO_API const char* ppo_last_error(void) { return g_err; }

// ---------------------------------------------------------------- profiler
// HIP events around the launches of the named kernels (comma-separated list),
// on the stream each launch goes to.
static char g_prof_names[1024] = "";
static int g_prof_cap = 0, g_prof_n = 0;
static hipEvent_t* g_ev0 = nullptr;
static hipEvent_t* g_ev1 = nullptr;
static double* g_work = nullptr;
static int* g_which = nullptr;   // index of the name in the list

static int prof_index(const char* name) {
  const size_t n = strlen(name);
  int idx = 0;
  for (const char* p = g_prof_names; *p;) {
    const char* e = strchr(p, ',');
    const size_t len = e ? (size_t)(e - p) : strlen(p);
    if (len == n && strncmp(p, name, n) == 0) return idx;
    if (!e) break;
    p = e + 1;
    ++idx;
  }
  return -1;
}

bool ppo_prof_begin(const char* name, hipStream_t st, int* slot) {
  if (g_prof_cap == 0 || g_prof_n >= g_prof_cap) return false;
  const int w = prof_index(name);
  if (w < 0) return false;
  *slot = g_prof_n++;
  g_which[*slot] = w;
  (void)hipEventRecord(g_ev0[*slot], st);
  return true;
}

void ppo_prof_end(int slot, hipStream_t st, double work) {
  (void)hipEventRecord(g_ev1[slot], st);
  g_work[slot] = work;
}

static void prof_free() {
  for (int i = 0; i < g_prof_cap; ++i) {
    (void)hipEventDestroy(g_ev0[i]);
    (void)hipEventDestroy(g_ev1[i]);
  }
  delete[] g_ev0;
  delete[] g_ev1;
  delete[] g_work;
  delete[] g_which;
  g_ev0 = g_ev1 = nullptr;
  g_work = nullptr;
  g_which = nullptr;
  g_prof_cap = g_prof_n = 0;
}

// names == NULL disables.  Not thread-safe; call outside captured regions.
PPO_API int ppo_prof_enable(const char* names, int capacity) {
  prof_free();
  if (!names || capacity <= 0) return 0;
  snprintf(g_prof_names, sizeof(g_prof_names), "%s", names);
  g_ev0 = new hipEvent_t[capacity];
  g_ev1 = new hipEvent_t[capacity];
  g_work = new double[capacity];
  g_which = new int[capacity];
  for (int i = 0; i < capacity; ++i) {
    PPO_HIP_CHECK(hipEventCreate(&g_ev0[i]), "ppo_prof_enable");
    PPO_HIP_CHECK(hipEventCreate(&g_ev1[i]), "ppo_prof_enable");
  }
  g_prof_cap = capacity;
  g_prof_n = 0;
  return 0;
}

// Waits for the recorded launches of the idx-th listed name (-1: all);
// out3 = {launches, Σ ms, Σ work}.
PPO_API int ppo_prof_collect_one(int idx, double* out3) {
  double ms_total = 0.0, work = 0.0;
  int n = 0;
  for (int i = 0; i < g_prof_n; ++i) {
    if (idx >= 0 && g_which[i] != idx) continue;
    PPO_HIP_CHECK(hipEventSynchronize(g_ev1[i]), "ppo_prof_collect");
    float ms = 0.f;
    PPO_HIP_CHECK(hipEventElapsedTime(&ms, g_ev0[i], g_ev1[i]), "ppo_prof_collect");
    ms_total += ms;
    work += g_work[i];
    ++n;
  }
  out3[0] = n;
  out3[1] = ms_total;
  out3[2] = work;
  return 0;
}

PPO_API int ppo_prof_collect(double* out3) { return ppo_prof_collect_one(-1, out3); }
PPO_API int ppo_abi_version(void) { return 3; }

namespace {

// insert (storage.py:62-73) for the per-env scalars; obs/vector_obs/hxs rows
// are bulk-copied with ppo_copy (or already written in place).
__global__ __launch_bounds__(256) void insert_scalars_kernel(
    int N, int step, const int64_t* __restrict__ action, const float* __restrict__ logp,
    const float* __restrict__ value, const float* __restrict__ reward, const float* __restrict__ mask,
    const float* __restrict__ bad_mask, int64_t* __restrict__ actions, float* __restrict__ action_log_probs,
    float* __restrict__ value_preds, float* __restrict__ rewards, float* __restrict__ masks,
    float* __restrict__ bad_masks) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const size_t t0 = (size_t)step * N + n, t1 = (size_t)(step + 1) * N + n;
  if (action) actions[t0] = action[n];
  if (logp) action_log_probs[t0] = logp[n];
  if (value) value_preds[t0] = value[n];
  if (reward) rewards[t0] = reward[n];
  if (mask) masks[t1] = mask[n];
  if (bad_mask) bad_masks[t1] = bad_mask[n];
}

// dst[i] = src[idx[i]] for rows of row_bytes (feed_forward_generator's
// `[indices]`, storage.py:143-157).  One wave per row, 16-B lanes.
template <typename V>
__global__ __launch_bounds__(256) void gather_rows_kernel(const V* __restrict__ src, const int64_t* __restrict__ idx,
                                                          V* __restrict__ dst, long long nrows, long long row_elems) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const V* s = src + idx[row] * row_elems;
  V* d = dst + row * row_elems;
  for (long long i = threadIdx.x & 63; i < row_elems; i += 64) d[i] = s[i];
}

// fp16 observation rows (RolloutStorage.half(), storage.py:48-58) -> fp32 rows for
// the conv1 loaders: dst[r] = (float)src[idx ? idx[r] : r], 8 halves per lane step.
__global__ __launch_bounds__(256) void gather_f16_f32_kernel(const uint4* __restrict__ src,
                                                             const int64_t* __restrict__ idx, float4* __restrict__ dst,
                                                             long long nrows, long long row_vec8) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const uint4* s = src + (idx ? idx[row] : row) * row_vec8;
  float4* d = dst + row * 2 * row_vec8;
  for (long long i = threadIdx.x & 63; i < row_vec8; i += 64) {
    const uint4 v = s[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    float f[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f[2 * q] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[q] & 0xFFFF));
      f[2 * q + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[q] >> 16));
    }
    d[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    d[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
  }
}

// Env-column gather for recurrent_generator (storage.py:181-205):
// dst[t][j] = src[t][envs[j]] for t < T, rows of row_bytes.
template <typename V>
__global__ __launch_bounds__(256) void gather_cols_kernel(const V* __restrict__ src, const int64_t* __restrict__ envs,
                                                          V* __restrict__ dst, int T, int N, int nsel,
                                                          long long row_elems) {
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (long long)T * nsel) return;
  const int t = (int)(r / nsel), j = (int)(r % nsel);
  const V* s = src + ((long long)t * N + envs[j]) * row_elems;
  V* d = dst + r * row_elems;
  for (long long i = threadIdx.x & 63; i < row_elems; i += 64) d[i] = s[i];
}

// Synthetic environment step: writes the next observation
// straight into its storage slot plus reward / done-mask planes.
//   obs byte  = byte k of mix64(seed ^ H(step, env, 8-byte block))
//   reward    = U(0,1]  from mix64(seed, step, env, 'r')
//   done      = U < p_done  -> mask 0, else 1; bad_mask = 1
__global__ __launch_bounds__(256) void synth_env_kernel(uint8_t* __restrict__ obs, int N, long long obs_bytes,
                                                        float* __restrict__ reward, float* __restrict__ mask,
                                                        float* __restrict__ bad_mask, uint64_t seed,
                                                        uint64_t step, float p_done) {
  const long long chunks = obs_bytes / 16;  // 16-B pieces per env
  const long long total = chunks * N;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long n = i / chunks, c = i % chunks;
    const uint64_t key = seed ^ mix64(step * 0x100000001B3ull + (uint64_t)n * 0x9E3779B1ull);
    const uint64_t h0 = mix64(key + (uint64_t)(2 * c));
    const uint64_t h1 = mix64(key + (uint64_t)(2 * c + 1));
    uint4 v;
    v.x = (uint32_t)h0;
    v.y = (uint32_t)(h0 >> 32);
    v.z = (uint32_t)h1;
    v.w = (uint32_t)(h1 >> 32);
    reinterpret_cast<uint4*>(obs + n * obs_bytes)[c] = v;
  }
  const long long n = (long long)blockIdx.x * 256 + threadIdx.x;
  if (n < N) {
    const uint64_t k = mix64(seed ^ mix64(step * 0x100000001B3ull + (uint64_t)n * 0x9E3779B1ull + 0x5EEDull));
    if (reward) reward[n] = u01_open0(k) - (1.0f / 16777216.0f);  // [0, 1)
    const float u = u01_open0(mix64(k ^ 0xD0D0D0D0ull));
    if (mask) mask[n] = (u < p_done) ? 0.0f : 1.0f;
    if (bad_mask) bad_mask[n] = 1.0f;
  }
}

// CartPole-v1 (gym's classic-control cart-pole, the c1 config's env; gym is not
// a dependency here, its published dynamics are restated): Euler integration at
// tau = 0.02, force ±10 N, termination at |x| > 2.4 or |θ| > 12°, reward 1 per
// step, TimeLimit 500 -> bad_transition (bad_mask 0), reset U(-0.05, 0.05)^4
// from the counter RNG, auto-reset as baselines' VecEnv does.  fp32 state
// (gym keeps float64 and returns float32 observations).
__global__ __launch_bounds__(256) void cartpole_kernel(float* __restrict__ state, int* __restrict__ steps,
                                                       const int64_t* __restrict__ action, float* __restrict__ obs,
                                                       float* __restrict__ reward, float* __restrict__ mask,
                                                       float* __restrict__ bad_mask, float* __restrict__ ep_len,
                                                       int N, uint64_t seed, uint64_t counter, int max_steps) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float* st = state + 4 * (size_t)n;
  bool reset = action == nullptr;
  float ended = 0.f;
  if (!reset) {
    const float gravity = 9.8f, masscart = 1.0f, masspole = 0.1f, total_mass = masspole + masscart;
    const float length = 0.5f, polemass_length = masspole * length, force_mag = 10.0f, tau = 0.02f;
    const float theta_thr = 12.0f * 2.0f * 3.14159265358979f / 360.0f, x_thr = 2.4f;
    float x = st[0], x_dot = st[1], theta = st[2], theta_dot = st[3];
    const float force = action[n] == 1 ? force_mag : -force_mag;
    const float ct = cosf(theta), sn = sinf(theta);
    const float temp = (force + polemass_length * theta_dot * theta_dot * sn) / total_mass;
    const float thetaacc = (gravity * sn - ct * temp) / (length * (4.0f / 3.0f - masspole * ct * ct / total_mass));
    const float xacc = temp - polemass_length * thetaacc * ct / total_mass;
    x = x + tau * x_dot;
    x_dot = x_dot + tau * xacc;
    theta = theta + tau * theta_dot;
    theta_dot = theta_dot + tau * thetaacc;
    st[0] = x; st[1] = x_dot; st[2] = theta; st[3] = theta_dot;
    const int k = ++steps[n];
    const bool done = x < -x_thr || x > x_thr || theta < -theta_thr || theta > theta_thr;
    const bool trunc = !done && k >= max_steps;
    if (reward) reward[n] = 1.0f;
    if (mask) mask[n] = (done || trunc) ? 0.0f : 1.0f;
    if (bad_mask) bad_mask[n] = trunc ? 0.0f : 1.0f;
    if (done || trunc) {
      ended = (float)k;
      reset = true;
    }
  }
  if (reset) {
    const uint64_t key = seed ^ mix64(counter * 0x100000001B3ull + (uint64_t)n * 0x9E3779B1ull + 0xCA27ull);
    for (int i = 0; i < 4; ++i) st[i] = (u01_open0(mix64(key + i)) - 0.5f) * 0.1f;
    steps[n] = 0;
  }
  if (ep_len) ep_len[n] = ended;
  for (int i = 0; i < 4; ++i) obs[4 * (size_t)n + i] = st[i];
}

__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ p, long long n, float v) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = v;
}

}  // namespace

PPO_API int ppo_copy(void* dst, const void* src, long long bytes, void* stream) {
  if (bytes <= 0 || dst == src) return 0;
  PPO_HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, as_stream(stream)), "ppo_copy");
  return 0;
}

PPO_API int ppo_fill_f32(float* p, long long n, float v, void* stream) {
  if (n <= 0) return 0;
  long long b = (n + 255) / 256;
  fill_f32_kernel<<<(unsigned)(b < 4096 ? b : 4096), 256, 0, as_stream(stream)>>>(p, n, v);
  PPO_LAUNCH_CHECK("fill_f32_kernel");
  return 0;
}

PPO_API int ppo_storage_insert_scalars(int N, int step, const int64_t* action, const float* logp, const float* value,
                                       const float* reward, const float* mask, const float* bad_mask,
                                       int64_t* actions, float* action_log_probs, float* value_preds,
                                       float* rewards, float* masks, float* bad_masks, void* stream) {
  PPO_REQUIRE(N > 0 && step >= 0, "ppo_storage_insert_scalars: N=%d step=%d", N, step);
  ProfScope prof("insert", as_stream(stream), 48.0 * N);
  insert_scalars_kernel<<<ceil_div(N, 256), 256, 0, as_stream(stream)>>>(
      N, step, action, logp, value, reward, mask, bad_mask, actions, action_log_probs, value_preds, rewards, masks,
      bad_masks);
  PPO_LAUNCH_CHECK("insert_scalars_kernel");
  return 0;
}

PPO_API int ppo_gather_rows(const void* src, const int64_t* idx, void* dst, long long nrows, long long row_bytes,
                            void* stream) {
  PPO_REQUIRE(nrows >= 0 && row_bytes > 0, "ppo_gather_rows: nrows=%lld row_bytes=%lld", nrows, row_bytes);
  if (nrows == 0) return 0;
  const unsigned blocks = ceil_div(nrows, 4);
  hipStream_t st = as_stream(stream);
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  if (row_bytes % 16 == 0 && al % 16 == 0)
    gather_rows_kernel<uint4><<<blocks, 256, 0, st>>>((const uint4*)src, idx, (uint4*)dst, nrows, row_bytes / 16);
  else if (row_bytes % 4 == 0 && al % 4 == 0)
    gather_rows_kernel<uint32_t><<<blocks, 256, 0, st>>>((const uint32_t*)src, idx, (uint32_t*)dst, nrows,
                                                         row_bytes / 4);
  else
    gather_rows_kernel<uint8_t><<<blocks, 256, 0, st>>>((const uint8_t*)src, idx, (uint8_t*)dst, nrows, row_bytes);
  PPO_LAUNCH_CHECK("gather_rows_kernel");
  return 0;
}

PPO_API int ppo_gather_f16_to_f32(const void* src, const int64_t* idx, float* dst, long long nrows,
                                  long long row_elems, void* stream) {
  PPO_REQUIRE(nrows >= 0 && row_elems > 0 && row_elems % 8 == 0, "ppo_gather_f16_to_f32: nrows=%lld row_elems=%lld",
              nrows, row_elems);
  PPO_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "ppo_gather_f16_to_f32: 16-B alignment");
  if (nrows == 0) return 0;
  gather_f16_f32_kernel<<<ceil_div(nrows, 4), 256, 0, as_stream(stream)>>>((const uint4*)src, idx, (float4*)dst,
                                                                           nrows, row_elems / 8);
  PPO_LAUNCH_CHECK("gather_f16_f32_kernel");
  return 0;
}

PPO_API int ppo_gather_env_columns(const void* src, const int64_t* envs, void* dst, int T, int N, int nsel,
                                   long long row_bytes, void* stream) {
  PPO_REQUIRE(T > 0 && N > 0 && nsel >= 0 && row_bytes > 0, "ppo_gather_env_columns: bad shape");
  if (nsel == 0) return 0;
  const unsigned blocks = ceil_div((long long)T * nsel, 4);
  hipStream_t st = as_stream(stream);
  const uintptr_t al = (uintptr_t)src | (uintptr_t)dst;
  if (row_bytes % 16 == 0 && al % 16 == 0)
    gather_cols_kernel<uint4><<<blocks, 256, 0, st>>>((const uint4*)src, envs, (uint4*)dst, T, N, nsel, row_bytes / 16);
  else if (row_bytes % 4 == 0 && al % 4 == 0)
    gather_cols_kernel<uint32_t><<<blocks, 256, 0, st>>>((const uint32_t*)src, envs, (uint32_t*)dst, T, N, nsel,
                                                         row_bytes / 4);
  else
    gather_cols_kernel<uint8_t><<<blocks, 256, 0, st>>>((const uint8_t*)src, envs, (uint8_t*)dst, T, N, nsel,
                                                        row_bytes);
  PPO_LAUNCH_CHECK("gather_cols_kernel");
  return 0;
}

PPO_API int ppo_synth_env_step(uint8_t* obs, int N, long long obs_bytes, float* reward, float* mask, float* bad_mask,
                               unsigned long long seed, unsigned long long step, float p_done, void* stream) {
  PPO_REQUIRE(N > 0 && obs_bytes > 0 && obs_bytes % 16 == 0, "ppo_synth_env_step: N=%d obs_bytes=%lld", N,
              obs_bytes);
  PPO_REQUIRE(((uintptr_t)obs & 15) == 0, "ppo_synth_env_step: obs not 16-B aligned");
  ProfScope prof("synth_env", as_stream(stream), (double)N * (obs_bytes + 12));
  long long work = (obs_bytes / 16) * N;
  long long b = (work + 255) / 256;
  long long bmin = (N + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < bmin) b = bmin;
  synth_env_kernel<<<(unsigned)b, 256, 0, as_stream(stream)>>>(obs, N, obs_bytes, reward, mask, bad_mask, seed, step,
                                                               p_done);
  PPO_LAUNCH_CHECK("synth_env_kernel");
  return 0;
}

PPO_API int ppo_cartpole_step(float* state, int* steps, const int64_t* action, float* obs, float* reward, float* mask,
                              float* bad_mask, float* ep_len, int N, unsigned long long seed,
                              unsigned long long counter, int max_steps, void* stream) {
  PPO_REQUIRE(N > 0 && max_steps > 0, "ppo_cartpole_step: N=%d max_steps=%d", N, max_steps);
  cartpole_kernel<<<ceil_div(N, 256), 256, 0, as_stream(stream)>>>(state, steps, action, obs, reward, mask, bad_mask,
                                                                   ep_len, N, seed, counter, max_steps);
  PPO_LAUNCH_CHECK("cartpole_kernel");
  return 0;
}
