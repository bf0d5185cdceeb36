/*
 * ppo_hip.h — C ABI of libppo_hip.so, the MI355X (gfx950) engine behind the
 * a2c_ppo_acktr Policy / RolloutStorage / PPO.update() API of ppo-dash.
 *
 * The reference has no native code and no FFI: its
 * boundary is the Python class API of ppo-dash-training/pytorch-a2c-ppo-acktr-gail/
 * a2c_ppo_acktr/{storage,model,distributions}.py and algo/ppo.py, and every
 * hot-path op is a stock PyTorch call.  Each entry point below replaces one of
 * those calls; the citation names the reference line it stands in for
 * (paths relative to that a2c_ppo_acktr/ directory).
 *
 * Conventions
 *   - every pointer is a device pointer owned by the caller (the library never
 *     allocates or frees caller memory); `stream` is a hipStream_t;
 *   - calls are asynchronous on `stream` and never synchronise the device (the
 *     two readers of device state, ppo_gru_persist_timeouts and the profiler's
 *     collect, wait for their own stream / events only);
 *   - kernel launches are safe from several host threads on distinct streams:
 *     the library's scratch (the persistent GRU's counters) is keyed by
 *     (device, stream), or passed in by the caller (ppo_gru_seq_fwd_ws).  The
 *     tuning knobs (ppo_tune_set, ppo_gru_*_set) and the profiler are
 *     process-global configuration: set them from one thread, between launches;
 *   - return 0 on success, a hipError_t or a PPO_E* code otherwise;
 *     ppo_last_error() returns the message of the calling thread's last error;
 *   - storage planes are [T(+1)][N] fp32 (time-major, env-minor), actions i64,
 *     observations u8 (or f32) [rows][C][84][84]; activations NHWC fp32.
 */
#ifndef PPO_HIP_H
#define PPO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPO_EARG 1001
#define PPO_ESHAPE 1002

const char* ppo_last_error(void);
/* 3 (round 6): symbols removed in round 5 (ppo_a1split_*, ppo_conv*_split, the anatomy
 * probes); round 6: ppo_gru_l2_set / _get removed (the BPTT hands dgh over by sc1 stores
 * only) and the GRU counter buffer is 2·G ints (ppo_gru_seq_counters) */
int ppo_abi_version(void);
/* launch-level event profiler used by bench.py: time every launch of the named
 * kernel (NULL disables); collect -> {launches, Σ ms, Σ algorithmic FLOP} */
int ppo_prof_enable(const char* names, int capacity);   /* comma-separated kernel names */
int ppo_prof_collect(double* out3);                       /* all listed: {launches, ms, work} */
int ppo_prof_collect_one(int idx, double* out3);          /* the idx-th listed name only */

/* ---------------- returns / advantages ------------------------------------ */
/* storage.py:82-121 RolloutStorage.compute_returns (all four branches,
 * bit-identical).  adv/partials (both or neither): also write
 * adv = returns[:-1] - value_preds[:-1] (algo/ppo.py:35) and per-block
 * (count, mean, M2) moment partials, 3*ppo_gae_partials_count(N) doubles. */
int ppo_gae_partials_count(int N);
int ppo_compute_returns(const float* rewards, float* value_preds, const float* masks, const float* bad_masks,
                        const float* next_value, float* returns, float* adv, double* partials, int T, int N,
                        double gamma, double gae_lambda, int use_gae, int use_proper_time_limits, void* stream);
/* time-parallel compute_returns (same arguments and side effects; within
 * tolerance, not bit-exact): each lane's affine recurrence folded per time chunk,
 * chunk carries composed through LDS — for few lanes / long T (c1, c2);
 * partials: 3*ppo_gae_scan_partials_count(N) doubles */
int ppo_gae_scan_partials_count(int N);
int ppo_compute_returns_scan(const float* rewards, float* value_preds, const float* masks, const float* bad_masks,
                             const float* next_value, float* returns, float* adv, double* partials, int T, int N,
                             double gamma, double gae_lambda, int use_gae, int use_proper_time_limits, void* stream);
/* algo/ppo.py:35 advantages = returns[:-1] - value_preds[:-1] (+ partials, 3 doubles per block) */
int ppo_adv_diff_partials_count(long long n);
int ppo_adv_diff(const float* returns, const float* value_preds, float* adv, double* partials, long long n,
                 void* stream);
/* algo/ppo.py:36 advantages.mean()/std(): stats = {count, mean, M2}, merged from the
 * block partials with Chan et al.'s update in a fixed order (Welford; ranks merge
 * their triples the same way, _dist.allreduce_stats); count is taken from the
 * partials (the argument is unused) */
int ppo_adv_finalize(const double* partials, int nparts, double count, double* stats, void* stream);
/* algo/ppo.py:36-37 (adv - mean) / (std + 1e-5), std unbiased */
int ppo_adv_normalize(float* adv, long long n, const double* stats, void* stream);

/* ---------------- rollout storage ----------------------------------------- */
/* storage.py:62-80 copy_ of bulk rows (insert / after_update) */
int ppo_copy(void* dst, const void* src, long long bytes, void* stream);
int ppo_fill_f32(float* p, long long n, float v, void* stream);
/* storage.py:66-71 insert of the per-env scalars; any source may be NULL */
int ppo_storage_insert_scalars(int N, int step, const int64_t* action, const float* logp, const float* value,
                               const float* reward, const float* mask, const float* bad_mask, int64_t* actions,
                               float* action_log_probs, float* value_preds, float* rewards, float* masks,
                               float* bad_masks, void* stream);
/* storage.py:143-157 feed_forward_generator `[indices]` row gathers */
int ppo_gather_rows(const void* src, const int64_t* idx, void* dst, long long nrows, long long row_bytes,
                    void* stream);
/* half-precision storage (storage.py:48-58 RolloutStorage.half()): fp16 observation
 * rows src[idx[r]] (idx NULL: row r) -> fp32 rows for the conv1 loaders */
int ppo_gather_f16_to_f32(const void* src, const int64_t* idx, float* dst, long long nrows, long long row_elems,
                          void* stream);
/* storage.py:181-205 recurrent_generator env-column stacking */
int ppo_gather_env_columns(const void* src, const int64_t* envs, void* dst, int T, int N, int nsel,
                           long long row_bytes, void* stream);
/* stands in for VecPyTorch.step + the simulator (make_env.py:58-114): u8 obs
 * written into the storage slot, reward U[0,1), done ~ Bernoulli(p_done) */
int ppo_synth_env_step(uint8_t* obs, int N, long long obs_bytes, float* reward, float* mask, float* bad_mask,
                       unsigned long long seed, unsigned long long step, float p_done, void* stream);

/* CartPole-v1 dynamics (c1's env, restated; gym absent): one step of every lane
 * (action NULL: reset), obs [N][4] written in place, auto-reset on done /
 * TimeLimit(max_steps) with bad_mask 0 on truncation; ep_len = finished length or 0 */
int ppo_cartpole_step(float* state, int* steps, const int64_t* action, float* obs, float* reward, float* mask,
                      float* bad_mask, float* ep_len, int N, unsigned long long seed, unsigned long long counter,
                      int max_steps, void* stream);

/* ---------------- CNNBase trunk (model.py:176-180) ------------------------- */
long long ppo_packed_weights_size(int H);
int ppo_packed_offsets(int H, long long* off6);
/* once per optimizer step: torch-layout conv2/conv3/fc weights -> loader orders; every packed f32
 * segment is followed by its exact bf16 split (hi, mid, lo planes), the B operand of the bf16 cores */
int ppo_pack_weights(const float* w2, const float* w3, const float* w4, int H, float* packed, void* stream);
/* model.py:177 Conv2d(C,32,8,s4)+ReLU over obs rows (idx: storage-row gather,
 * storage.py:143; NULL: rows row0..row0+B-1); u8 staged as integers, 1/255 applied
 * to the accumulator (Σ w·u/255) */
int ppo_conv1_fwd(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B, const float* w1,
                  const float* b1, float* out, void* stream);
/* the same, also writing the ReLU mask of `out` as bits for the backward pass
 * (mbits [B][400] u32: bit c of pixel p = out[p][c] > 0, 1.6 KB per image) */
int ppo_conv1_fwd_mask(const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C, int B,
                       const float* w1, const float* b1, float* out, uint32_t* mbits, void* stream);
/* conv1 on the observation forms of the reference's own env chain (conv1f.hip):
 * image-resident split-bf16 MFMA kernels (both operands split three ways, six part
 * products: fp32 accuracy).  ppo_conv1_fwd / ppo_conv1_wgrad route fp32
 * observations with C = 4 here.  mbits (nullable): ReLU mask bits as
 * ppo_conv1_fwd_mask writes them.
 *   _f32: fp32 rows [4][84][84] (the fp32 storage plane T/run.py fills,
 *         storage.py:12), 16-B aligned;
 *   _rgb: raw u8 RGB frames [84][84][3] (21,168 B rows, 16-B aligned) decoded in
 *         the operand loader exactly as NormalizeWrapper + FrameStackMono(2) +
 *         TransposeImage + .float() (T/sohojoe_wrappers.py:958-991, 563-638;
 *         T/make_env.py:411-413; = ppo_obs_preprocess mode 2 / 1 / 0 with mono):
 *         channel c < 3 = fl32(((double)u - mean[y][x][c]) / std), channel 3 the
 *         transposed grey plane; mean fp32 [84][84][3] (NULL: 0; then std 255
 *         gives u/255, std 1 the raw values — raw mode, where the frame is still
 *         u8 inside FrameStackMono and its grey plane is stored truncated to u8).  Weight gradients: split-K slab
 *         [Z][32][256] + bias partials [Z][32] (reduce with scale 1).
 *         Default (ppo_tune_set("rgb_aff", 1), every mode but raw): the affine fold
 *         (rgbaff.hip) — conv1 of the decoded input as rs * (exact u8 MFMA sums over
 *         the colour planes at the direct and the transposed patch origin, grey
 *         weights folded in) + the means' per-pixel bias map; fp32-accurate but not
 *         bit-identical to the decode chain.  rgb_aff 0: the bit-exact fused decode. */
int ppo_conv1_fwd_f32(const float* obs, const int64_t* idx, long long row0, int B, const float* w1, const float* b1,
                      float* out, uint32_t* mbits, void* stream);
int ppo_conv1_fwd_rgb(const uint8_t* frames, const int64_t* idx, long long row0, int B, const float* mean, double stdv,
                      const float* w1, const float* b1, float* out, uint32_t* mbits, void* stream);
int ppo_conv1_wgrad_f32(const float* dz1, const float* obs, const int64_t* idx, long long row0, int B, int Z,
                        float* slab, float* slab_bias, void* stream);
int ppo_conv1_wgrad_rgb(const float* dz1, const uint8_t* frames, const int64_t* idx, long long row0, int B,
                        const float* mean, double stdv, int Z, float* slab, float* slab_bias, void* stream);
/* model.py:178 Conv2d(32,64,4,s2)+ReLU */
int ppo_conv2_fwd(const float* a1, int B, const float* w2p, const float* b2, float* out, void* stream);
/* the same, also writing its ReLU mask as bits (mbits [B][81] u64: bit c of pixel p = out[p][c] > 0) */
int ppo_conv2_fwd_mask(const float* a1, int B, const float* w2p, const float* b2, float* out, uint64_t* mbits,
                       void* stream);
/* model.py:179 Conv2d(64,32,3,s1)+ReLU */
int ppo_conv3_fwd(const float* a2, int B, const float* w3p, const float* b3, float* out, void* stream);
/* conv1 -> conv2 -> conv3 forward of u8 4-channel observation rows (model.py:177-179) in
 * one persistent launch: a1 / a2 / a3 bit-identical to ppo_conv1_fwd, ppo_conv2_fwd and
 * ppo_conv3_fwd; m1 / m2 both NULL or both given (the ReLU mask bits of
 * ppo_conv1_fwd_mask / ppo_conv2_fwd_mask).  Replaces the trunk's three launches
 * (model.py:177-179 as one call). */
int ppo_trunk_fwd(const uint8_t* obs, const int64_t* idx, long long row0, int B, const float* w1, const float* b1,
                  float* a1, uint32_t* m1, const float* w2p, const float* b2, float* a2, uint64_t* m2,
                  const float* w3p, const float* b3, float* a3, void* stream);
/* model.py:180 Linear(1568,H)+ReLU (generic Linear+ReLU) */
/* model.py:181 CNNBase fc + ReLU from the packed W4p segment (ppo_pack_weights; its bf16 planes follow it):
 * out[m * ldo + n] = relu(x[m] · W4p[n] + b[n]), x [M][1568] (p, c) order */
int ppo_fc_fwd(const float* x, int M, const float* w4p, const float* b, int H, float* out, int ldo, void* stream);
/* the same with a caller-owned workspace: rollout-sized M (M * H <= 4096 * 1024) runs
 * split-K (ppo_tune_set("fc_splitk", Z) slices, default 2) into ws and a fixed-order
 * reduce + bias + ReLU; ws_bytes below ppo_fc_fwd_ws_bytes(M, H) (0: no split) falls
 * back to ppo_fc_fwd */
long long ppo_fc_fwd_ws_bytes(int M, int H);
int ppo_fc_fwd_ws(const float* x, int M, const float* w4p, const float* b, int H, float* out, int ldo, float* ws,
                  long long ws_bytes, void* stream);
int ppo_linear_relu_fwd(const float* x, int M, int K, const float* w, const float* b, int N, float* out,
                        void* stream);
/* Linear with row strides, optional A-row gather, bias and activation
 * (0 none, 1 ReLU, 2 tanh): the fc into a padded [x | vector_obs] row, the GRU
 * input projection, MLPBase's tanh layers (model.py:212-218) */
int ppo_linear_fwd_ex(const float* x, const int64_t* idx, int M, int K, int lda, const float* w, const float* b,
                      int N, float* out, int ldo, int act, void* stream);
/* dgrad through the activation that produced `act` (mode 1 ReLU, 2 tanh) */
int ppo_linear_dgrad_ex(const float* dy, int M, int K, const float* wt, int N, const float* act, int ldact, int mode,
                        float* dx, void* stream);
/* dst [cols][rows] = srcᵀ */
int ppo_transpose(const float* src, int rows, int cols, float* dst, void* stream);
/* algo/ppo.py:80-81 loss.backward() through the trunk: dgrad with the ReLU mask
 * of the layer below fused, wgrad as split-K partial slabs + deterministic reduce */
int ppo_linear_dgrad_mask(const float* dy, int M, int K, const float* wt, int N, const float* act, float* dx,
                          void* stream);
/* the training forward's conv3 (model.py:179) that also writes its ReLU mask bits,
 * uint16 [B][49][2] (bit j of word (p, t): output channel 16 t + j of pixel p > 0), and
 * the fc dgrad (N = 1568) masked by those bits instead of the fp32 activation:
 * bit-identical to ppo_conv3_fwd + ppo_linear_dgrad_mask(act = conv3's output) */
int ppo_conv3_fwd_mask(const float* a2, int B, const float* w3p, const float* b3, float* out, uint16_t* mbits,
                       void* stream);
int ppo_fc_dgrad_bits(const float* dy, int M, int K, const float* wt, const uint16_t* mbits, float* dx,
                      void* stream);
int ppo_conv3_dgrad(const float* dz3, int B, const float* w3d, const float* a2, float* dz2, void* stream);
/* conv3 dgrad with conv2's ReLU mask as bits (from ppo_conv2_fwd_mask): 648 B instead of
 * 20.7 KB read per image; ppo_conv3_dgrad_bits_ok() is 1 (kept for ABI stability) */
int ppo_conv3_dgrad_bits_ok(void);
int ppo_conv3_dgrad_bits(const float* dz3, int B, const float* w3d, const uint64_t* m2bits, float* dz2,
                         void* stream);
int ppo_conv2_dgrad(const float* dz2, int B, const float* w2d, const float* a1, float* dz1, void* stream);
/* conv2 dgrad with conv1's ReLU mask as bits (from ppo_conv1_fwd_mask) instead of
 * the fp32 activations: 1.6 KB instead of 51.2 KB read per image;
 * ppo_conv2_dgrad_bits_ok() is 1 (kept for ABI stability) */
int ppo_conv2_dgrad_bits_ok(void);
int ppo_conv2_dgrad_bits(const float* dz2, int B, const float* w2d, const uint32_t* m1bits, float* dz1,
                         void* stream);
int ppo_wgrad_splits(long long R, int tiles, int target_blocks, int min_ktiles);
int ppo_conv1_wgrad(const float* dz1, const void* obs, int obs_is_u8, const int64_t* idx, long long row0, int C,
                    int B, int Z, float* slab, float* slab_bias, void* stream);
int ppo_conv2_wgrad(const float* dz2, const float* a1, int B, int Z, float* slab, float* slab_bias, void* stream);
int ppo_conv3_wgrad(const float* dz3, const float* a2, int B, int Z, float* slab, float* slab_bias, void* stream);
int ppo_linear_wgrad(const float* dy, const float* x, int R, int N, int K, int Z, float* slab, float* slab_bias,
                     void* stream);
/* CU-contention probe (probe.hip; diagnostics, not on the training path): `blocks`
 * workgroups that each spin for `ticks` of the 100 MHz s_memrealtime counter and record
 * (start, end) into stamps [blocks][2]; ppo_probe_now writes the counter's current value */
int ppo_probe_side_kernel(int blocks, int threads, long long ticks, long long* stamps, void* stream);
int ppo_probe_now(long long* out, void* stream);
/* scale multiplies the weight sums only (conv1 with u8 observations stages the
 * bytes as integers: pass 1/255); bias sums are unscaled */
int ppo_wgrad_reduce(const float* slab, const float* slab_bias, int Z, int M, int NW, int kind, int a, int b,
                     float* gw, float* gb, float scale, int accumulate, void* stream);
/* deterministic column sums out[c] = scale·Σ_r src[r*ld + c] (split-partial reduces) */
int ppo_colsum(const float* src, long long ld, int rows, long long cols, float* out, float scale, int accumulate,
               void* stream);
/* run-time knobs (A/B and test hooks; each key takes the listed values, any other
 * value is refused with PPO_EARG):
 *   "products"    part products per operand pair of the split-bf16 fp32 GEMMs of the
 *                 conv / fc kernels: 6 (default: dropped terms < 2^-26 |a·b|), 9 (every
 *                 product exact), 1 (the half-precision mode's one bf16 product).  The
 *                 GRU's W_hh products (H >= 128) always take 6 (fp32 MFMA at H = 64)
 *   "conv1_fwd"   0 image-resident kernel (default), 9 the generic tile GEMM
 *   "conv1_wgrad" 9 one-wave-per-SIMD k-split kernel (default), 10 its wave-pair form,
 *                 8 the eight-wave k-split kernel, 5 the part-pipelined kernel
 *   "x9"          1 split-bf16 dense GEMMs (default), 0 fp32 MFMA, 2 split everywhere
 *   "fc_splitk"   K slices of the rollout-sized fc forward, 0..8 (default 4)
 *   "fc_splitk_tile" 1 that fc on 128 x 128 tiles with 16-B slab stores (default), 0 on
 *                 128 x 64 tiles (bit-identical results for the same slice count)
 *   "rgb_aff"     1 affine-folded raw RGB conv1 (default), 0 bit-exact decode
 *   "stagger"     schedule bits 0..15 (default 2; every value gives the same results);
 *                 larger values are refused (they select timing-anatomy paths that give
 *                 wrong results by design, accepted only by a -DPPO_DIAG build)
 *   "small_b"     forwards of at most this many samples take small.hip's kernels (>= 0)
 *   "heads_lds"   0 / non-zero: the LDS-weight heads_train kernel off / on (default on) */
int ppo_tune_set(const char* key, int value);
/* current value of a tune key (-1 if unknown) */
int ppo_tune_get(const char* key);

/* ---------------- observation boundary ------------ */
/* NormalizeWrapper (ppo-dash-study/013_…/sohojoe_wrappers.py:872-884) +
 * FrameStackMono(k=2) (:425-501) + TransposeImage (pytorch_wrappers.py:170-203)
 * + VecPyTorch .float() (:105-160), fused: src u8 [N][S][S][3] RGB frames (env
 * stride src_stride bytes) -> dst fp32 [N][3 (+1 mono)][S][S] (env stride
 * dst_stride floats).  mode 0: raw values, 1: u8/255, 2: (u8 - mean[S][S][3]) / std
 * (float64 arithmetic, as numpy, then rounded to fp32).  mono: append the
 * reference's (transposed) cv2 RGB2GRAY channel. */
int ppo_obs_preprocess(const uint8_t* src, long long src_stride, int N, int S, int mode, const double* mean,
                       double stdv, int mono, float* dst, long long dst_stride, void* stream);
/* VecPyTorchFrameStack.step_wait / reset (pytorch_wrappers.py:58-102) on
 * stacked [N][nstack][frame_elems]: shift one frame left, zero envs with done[n]
 * (u8, nullable), write obs [N][frame_elems] into the last slot; reset = 1 zeroes
 * every slot first */
int ppo_frame_stack(float* stacked, int N, int nstack, long long frame_elems, const float* obs,
                    const uint8_t* done, int reset, void* stream);

/* ---------------- GRU (model.py:89-95, 111-166) ---------------------------- */
/* one step h' = GRU(gi, h_prev·mask) with the cell fused into the W_hh GEMM;
 * save_* (all or none) keep r, z, n, W_hn·h+b_hn, h_in for the backward */
int ppo_gru_step_fwd(const float* hprev, const float* masks, const int64_t* mask_idx, const float* whh,
                     const float* bhh, const float* gi, int M, int H, float* hout, float* save_r, float* save_z,
                     float* save_n, float* save_ghn, float* save_hin, void* stream);
/* backward of one step: gate gradients (dgi, dgh rows [M][3H]) and dh'·z */
int ppo_gru_cell_bwd(const float* dout, const float* carry, const float* r, const float* z, const float* n,
                     const float* ghn, const float* hin, float* dgi, float* dgh, float* dhz, int M, int H,
                     int has_carry, void* stream);
/* carry(t-1) = (dgh·W_hh + dh'·z)·mask(t) */
int ppo_gru_step_bwd(const float* dgh, const float* whhT, const float* dhz, const float* masks,
                     const int64_t* mask_idx, float* carry, int M, int H, void* stream);
/* W_ih -> zero-padded [3H][Ip], W_ih[:, :H]ᵀ [H][3H], W_hhᵀ [H][3H] */
/* step-kernel variant (A/B knob): 0 register-tiled 16x16x4 f32 MFMA kernels
 * (H in {64,128,256,512}), 1 the tile-GEMM steps */
int ppo_gru_variant_set(int v);
int ppo_gru_variant_get(void);
/* the BPTT loop body in one launch: step t's carry = (dgh(t)·W_hh + dhz)·m(t)
 * (ppo_gru_step_bwd) fused with step t-1's gate backward from that carry
 * (ppo_gru_cell_bwd with dout(t-1) and the saves of t-1; writes dgi/dgh of t-1
 * and overwrites dhz with t-1's).  H in {64, 128, 256, 512}, variant 0 only. */
/* whole-sequence forward / backward through time (one call per minibatch; the
 * per-step kernels above, launched from C): model.py:116-165 */
int ppo_gru_seq_fwd(const float* h0, const float* masks, const int64_t* idx, const float* whh, const float* bhh,
                    const float* gi, int T, int n, int H, float* hout, float* save_r, float* save_z, float* save_n,
                    float* save_ghn, float* save_hin, void* stream);
/* ppo_gru_seq_fwd runs as ONE persistent launch when ceil(n/32)·H/16 blocks fit
 * one per CU (H in {64,128,256,512}, variant 0): row groups hand h(t) over with
 * write-through stores and relaxed agent-scope counters, every wait bounded;
 * bit-identical to the step launches.  ppo_gru_seq_bwd likewise (persist bit 1).
 * persist: bit 0 forward, bit 1 backward (default 3); 0 forces the step launches.
 * Co-residency of the grid is assumed from its size, which holds on an unshared
 * device; when another process holds CUs a wait may run out: the launch then
 * sets its error word and every block returns without computing further steps
 * (fail-safe, not a hang).  With the library-held words (ppo_gru_seq_fwd) the
 * word is read by ppo_gru_persist_timeouts(stream); with ppo_gru_seq_fwd_ws the
 * caller owns it (sticky until the caller clears it; a launch that starts with
 * it set returns at once) and passes it to ppo_clip_adam_guarded. */
int ppo_gru_persist_set(int v);
int ppo_gru_persist_get(void);
/* polls before a bounded wait gives up (default 2^21; 0: every wait gives up at once —
 * the tests force timeouts with it) */
int ppo_gru_persist_spin_set(int polls);
/* 1 if a ppo_gru_seq_fwd launch on `stream` timed out since the last call (its
 * results are invalid), 0 if not, -1 on error; waits for `stream` only (a
 * stream-ordered read of the word) and clears it */
int ppo_gru_persist_timeouts(void* stream);
/* counters a persistent launch over n rows needs (ints; G = ceil(n/32) groups):
 * [G step counters][G BPTT reports: 1 the group ran the persistent BPTT (dgh handed
 * over by sc1 stores and loads), 0 not run] */
int ppo_gru_seq_counters(int n);
/* ppo_gru_seq_fwd with caller-owned synchronisation words: counters
 * (ppo_gru_seq_counters(n) ints, reset by the call on `stream`) and err (one int,
 * see above); both may be NULL when the step launches run (persist 0) */
int ppo_gru_seq_fwd_ws(const float* h0, const float* masks, const int64_t* idx, const float* whh, const float* bhh,
                       const float* gi, int T, int n, int H, float* hout, float* save_r, float* save_z,
                       float* save_n, float* save_ghn, float* save_hin, int* counters, int* err, void* stream);
int ppo_gru_seq_bwd(const float* dout, const float* save_r, const float* save_z, const float* save_n,
                    const float* save_ghn, const float* save_hin, const float* masks, const int64_t* idx,
                    const float* whhT, int T, int n, int H, float* dgi, float* dgh, float* dhz, float* carry,
                    void* stream);
/* ppo_gru_seq_bwd with caller-owned synchronisation words (as ppo_gru_seq_fwd_ws):
 * T > 1 runs step T-1's cell backward, then steps T-1 .. 1 as ONE persistent
 * launch (gru_seq_bwd16_kernel: W_hh^T slices resident, row groups hand dgh over
 * through write-through stores and counters; bounded waits set *err, sticky, and
 * ppo_clip_adam_guarded skips the optimizer step while it is set).  Results equal
 * the per-step launches (ppo_gru_persist_set(0)) bit for bit.  Replaces the BPTT of
 * torch.nn.GRU's autograd over T/a2c_ppo_acktr/model.py:116-165. */
int ppo_gru_seq_bwd_ws(const float* dout, const float* save_r, const float* save_z, const float* save_n,
                       const float* save_ghn, const float* save_hin, const float* masks, const int64_t* idx,
                       const float* whhT, int T, int n, int H, float* dgi, float* dgh, float* dhz, float* carry,
                       int* counters, int* err, void* stream);
int ppo_gru_step_bwd_cell(const float* dgh, const float* whhT, float* dhz, const float* masks,
                          const int64_t* mask_idx, float* carry, int M, int H, const float* dout_prev,
                          const float* r, const float* z, const float* n, const float* ghn, const float* hin,
                          float* dgi_prev, float* dgh_prev, void* stream);
int ppo_gru_pack(const float* wih, const float* whh, int H, int I, int Ip, float* wih_pad, float* wihT, float* whhT,
                 void* stream);
/* model.py:195 torch.cat((x, vector_inputs)): dst[r][col0 + c] = src[idx(r)][c], zero pad */
int ppo_concat_cols(const float* src, const int64_t* idx, long long rows, int ncols, float* dst, int ld, int col0,
                    int zero_to, void* stream);
/* storage.py:195-220 recurrent minibatch sample order: idx[t*n + j] = t*N + envs[j] */
int ppo_rec_indices(const int64_t* envs, int n, int T, int N, int64_t* idx, void* stream);

/* ---------------- heads, distribution, loss -------------------------------- */
/* model.py:54-79 act / get_value / evaluate_actions heads + distributions.py:17-27
 * FixedCategorical: value, logits, logsumexp, sample = argmax(probs/E) (noise =
 * E, host replay) or counter-RNG Exp(1) (noise NULL), mode, log_probs, entropy.
 * feat_v: critic features when they differ from the policy features (MLPBase,
 * model.py:231-234); NULL = feat */
int ppo_heads_act(const float* feat, const float* feat_v, int N, int H, const float* wc, const float* bc,
                  const float* wa,
                  const float* ba, int A, const float* noise, unsigned long long seed, unsigned long long counter,
                  int deterministic, const int64_t* given, float* value, int64_t* action, float* logp,
                  float* entropy, void* stream);
/* algo/ppo.py:57-81 evaluate_actions + clipped surrogate + clipped value loss +
 * entropy, forward and analytic backward to dL/dfeature (through the features'
 * activation feat_act: 0 none, 1 ReLU, 2 tanh), head-gradient partials; with
 * feat_v the critic branch's gradient goes to dfeat_v.  part_loss holds 4 floats
 * per block and loss_acc 4 doubles: {value loss, action loss, entropy, number of
 * stored actions outside [0, A)} — the last is where the reference's
 * log_probs gather raises (distributions.py:22); PPO.update raises on it.
 * ppo_heads_act with `given` writes a NaN log-prob for such a row. */
int ppo_heads_train_blocks(int B);
int ppo_heads_train(const float* feat, const float* feat_v, int B, int H, const float* wc, const float* bc,
                    const float* wa,
                    const float* ba, int A, const int64_t* idx, long long row0, const int64_t* actions,
                    const float* old_logp, const float* adv, const float* vpred, const float* ret, float clip,
                    float value_coef, float entropy_coef, float inv_b, int use_clipped_value_loss, int feat_act,
                    float* dfeat, float* dfeat_v, float* part_w, float* part_b, float* part_loss, void* stream);
int ppo_heads_reduce(const float* part_w, const float* part_b, const float* part_loss, int nblk, int H, int A,
                     float* g_wc, float* g_bc, float* g_wa, float* g_ba, double* loss_acc, double inv_b, float scale,
                     int use_clipped_value_loss, void* stream);
/* model.py:77 dist.entropy().mean() */
int ppo_mean_f32(const float* x, long long n, float* out, void* stream);

/* ---------------- clip + Adam (algo/ppo.py:82-84) -------------------------- */
int ppo_grad_partials_count(long long n);
int ppo_grad_sumsq(const float* g, long long n, float scale, double* partials, void* stream);
int ppo_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, long long n,
                  const double* partials, float scale, double max_norm, double lr, double beta1, double beta2,
                  double eps, long long step, double* norm_out, void* stream);
/* the same step, skipped when a guard is set: *guard_i != 0 (the persistent GRU's
 * error word) or *guard_d > 0 (loss_acc[3], stored actions outside [0, A) — where
 * the reference raises before its optimizer step, distributions.py:22); a skipped
 * step leaves params, grads and moments bit-unchanged and adds 1 to *skipped.
 * Any guard pointer may be NULL. */
int ppo_clip_adam_guarded(float* params, float* grads, float* exp_avg, float* exp_avg_sq, long long n,
                          const double* partials, float scale, double max_norm, double lr, double beta1,
                          double beta2, double eps, long long step, double* norm_out, const int* guard_i,
                          const double* guard_d, int* skipped, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PPO_HIP_H */
