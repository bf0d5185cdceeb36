#!/usr/bin/env python3
"""Benchmark: env-steps/s of the full PPO iteration (rollout + GAE + update),
BASELINE.json configs[2]: CNNBase (H=512), 4096 env lanes x 128 steps per GPU,
PPO 3 epochs x 8 minibatches, synthetic 84x84x4 u8 observations.

One bench "step" = one whole T/run.py:168-248 iteration on every rank:
  128 x (Policy.act -> synthetic env step -> RolloutStorage.insert),
  get_value, compute_returns (GAE), PPO.update (24 minibatches of fwd + bwd +
  [RCCL grad all-reduce] + clip + Adam), after_update.
value = envs_per_gpu * 128 * world * K / max-over-ranks(wall time of K steps).

Multi-GPU, one rank per GPU: env lanes are sharded (weak scaling); each
minibatch's flat gradient is all-reduced over RCCL.  Either launched by
torch.distributed.run (RANK / WORLD_SIZE in the environment; WORLD_SIZE must
equal --gpus), or, with `--gpus N` and no launcher, this script starts the N
ranks itself as child processes before anything touches the GPU.

Also reported on rank 0:
  roofline      the dominant kernel's achieved FLOP/s from HIP events recorded
                around each of its launches during the timed region
  gae_roofline  fused GAE + advantage kernel on a 1M-lane buffer (> Infinity Cache)
  cpu_baseline  the reference's CPU path restated in torch (oracle/torch_ref.py:
                F.conv2d / linear, autograd, torch.optim.Adam, clip_grad_norm_),
                timed on a bounded sample at 1 thread (T/run.py:55) and at the
                host's core share, CPU model named
  kernel_rooflines  every HIP kernel family of the iteration with its own
                roofline; the MFMA trunk kernels are event-timed inside the timed
                region, the rest in one extra profiled iteration after it
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "ppo-dash_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec (rollout+GAE+PPO update) at 4096 envs×128 steps, 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 MFMA = vector peak (dense)
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
PEAK_HBM_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
NOMINAL_SCLK_GHZ = 2.4          # the shader clock the MFMA peaks are quoted at

# Every HIP kernel family of the iteration and the roofline that bounds it
# (DESIGN.md §5): name (as the library's event profiler tags the launch) ->
# (bound, peak, work unit of the tag, instructions).  Work is algorithmic:
# fp32 FLOP = 2·M·N·K of the layer for the GEMMs, compulsory HBM bytes for the
# byte movers.  The split-bf16 kernels execute P bf16 part products per fp32
# product on the matrix cores — 3 with a u8 operand (exact in bf16), 6 (default)
# or 9 (ppo_tune_set("products")) with two fp32 operands — so their MFMA
# ceiling is the dense bf16 peak / P in fp32-FLOP units.
def profiled(products):
    split = (f"v_mfma_f32_16x16x32_bf16 x{products} "
             + {9: "(exact split)", 6: "(split, 6 products: fp32-accurate)",
                1: "(half-precision mode: bf16 operands)"}[products])
    pk = PEAK_BF16_MFMA_TFLOPS / products
    u8 = 1 if products == 1 else 3   # conv1: weight parts against the exact u8 pixels

    def mf(how):
        return ("mfma", pk, "flop", split + how)

    def hbm(how):
        return ("hbm", PEAK_HBM_GBPS, "bytes", how)
    return {
        "conv2_fwd": mf(", image-resident"),
        "conv2_dgrad": mf(", image-resident"),
        "conv2_wgrad": mf(", image-resident, ds_read_b64_tr_b16 im2col"),
        "conv3_fwd": mf(", image-resident"),
        "conv3_dgrad": mf(", image-resident"),
        "conv3_wgrad": mf(", image-resident, ds_read_b64_tr_b16 im2col"),
        # u8 pixels are exact in bf16: 3 products per fp32 product
        "conv1_wgrad_u8": ("mfma", PEAK_BF16_MFMA_TFLOPS / u8, "flop",
                           f"v_mfma_f32_32x32x16_bf16 x{u8} (u8 exact), image-resident"),
        # conv1 forward: 79,424 B of compulsory HBM traffic per sample (28,224 B u8 in, 51,200 B f32 out)
        # against 6.55 MFLOP at bf16/3 -> HBM-bound
        "conv1_fwd_u8": ("hbm", PEAK_HBM_GBPS, "conv1_flop", "v_mfma_f32_16x16x32_bf16 x3 (u8 exact), image-resident"),
        # --obs f32 / rgb: conv1 over fp32 operands (both split): the split MFMA ceiling
        "conv1_fwd_f32": mf(", conv1 on fp32 observation rows, image-resident parts"),
        "conv1_fwd_rgb": mf(", conv1 on raw RGB frames, NormalizeWrapper + FrameStackMono(2) decode fused"),
        "conv1_wgrad_f32": mf(", conv1 weight gradient on fp32 observation rows"),
        "conv1_wgrad_rgb": mf(", conv1 weight gradient on raw RGB frames, decode fused"),
        "obs_preprocess": hbm("f2 chain into the fp32 storage slot (--obs f32 env step)"),
        "fc_fwd": mf(", fc 1568->H + ReLU (tile GEMM)"),
        "linear_dgrad_mask": mf(", fc dgrad with conv3's ReLU mask"),
        "linear_wgrad": mf(", fc / GRU weight gradients, split-K slabs"),
        "linear_fwd_ex": mf(", GRU input projection / MLP layers"),
        "linear_dgrad_ex": mf(", GRU input dgrad / MLP layers"),
        # the GRU's W_hh products: split-bf16 x6 for H >= 128 (c5: H = 256); fp32 MFMA at H = 64
        "gru_seq_fwd": mf(", W_hh products of the persistent GRU forward (cell fused)"),
        "gru_seq_bwd": mf(", W_hh products of the persistent BPTT (gate backward fused)"),
        # the rollout's conv1 -> conv2 -> conv3 in one launch (conv1's share at x3 counted at x6: conservative)
        "trunk_fwd": mf(", rollout trunk conv1 -> conv2 -> conv3 as one persistent launch"),
        "heads_train": hbm("Categorical + PPO loss + analytic backward fused, one wave per row"),
        "heads_act": hbm("value / logits / Categorical sample fused"),
        "heads_reduce": hbm("head-gradient partial sums"),
        "wgrad_reduce": hbm("split-K slab reduce into the flat gradient"),
        "gae": hbm("GAE + advantage difference + moment partials"),
        "adv_norm": hbm("advantage normalisation"),
        "insert": hbm("RolloutStorage.insert scalars"),
        "synth_env": hbm("synthetic env: u8 frames written into the storage slot"),
        "grad_sumsq": hbm("clip_grad_norm_ partial sums"),
        "clip_adam": hbm("clip + Adam"),
        "pack_weights": hbm("per-step weight repack + bf16 split"),
    }


# event-timed inside the timed region (the MFMA trunk kernels; the dominant one
# is the `roofline` line); the rest are timed in one profiled iteration after it
TIMED = ("conv2_fwd", "conv2_dgrad", "conv2_wgrad", "conv3_fwd", "conv3_dgrad", "conv3_wgrad", "conv1_wgrad_u8",
         "conv1_fwd_u8", "conv1_fwd_f32", "conv1_wgrad_f32", "conv1_fwd_rgb", "conv1_wgrad_rgb")
PROFILED = profiled(6)
# compulsory HBM bytes per image of the image-resident conv kernels (fp32 NHWC
# activations, u8 observations, ReLU mask bits) and the layer's MACs per image:
# these kernels are MFMA- and HBM-heavy at once (conv1 wgrad reads 79 KB per
# image for 3.3 M MACs), so both rooflines are reported
CONV_HBM = {
    "conv1_fwd_u8": (3276800, 28224 + 51200),
    "conv1_fwd_f32": (3276800, 112896 + 51200),         # fp32 rows in, a1 out
    "conv1_fwd_rgb": (3276800, 21168 + 51200),          # raw RGB frame in, a1 out
    "conv1_wgrad_f32": (3276800, 51200 + 112896),
    "conv1_wgrad_rgb": (3276800, 51200 + 21168),
    "conv1_wgrad_u8": (3276800, 51200 + 28224),          # dz1 + u8 image
    "conv2_fwd": (2654208, 51200 + 20736),               # a1 + a2 (+ 648 B mask bits, training)
    "conv2_dgrad": (2654208, 20736 + 1600 + 51200),      # dz2 + conv1 mask bits + dz1
    "conv2_wgrad": (2654208, 20736 + 51200),             # dz2 + a1
    "conv3_fwd": (903168, 20736 + 6272),
    "conv3_dgrad": (903168, 6272 + 648 + 20736),
    "conv3_wgrad": (903168, 6272 + 20736),
}
CONV1_FWD_BYTES_PER_FLOP = 79424.0 / (2.0 * 400 * 32 * 256)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--envs", type=int, default=4096, help="env lanes per GPU")
    p.add_argument("--num-steps", type=int, default=128)
    p.add_argument("--ppo-epoch", type=int, default=3)
    p.add_argument("--num-mini-batch", type=int, default=8)
    p.add_argument("--hidden", type=int, default=None, help="default 512 (CNN) / 256 (GRU)")
    p.add_argument("--recurrent", action="store_true", help="c5: GRU policy + vector obs")
    p.add_argument("--vec-len", type=int, default=14, help="vector obs length with --recurrent (OTC v7: 14)")
    p.add_argument("--profile-kernels", default=",".join(TIMED),
                   help="kernels event-timed inside the timed region; the one with the most time is the roofline kernel")
    p.add_argument("--no-profile-pass", action="store_true",
                   help="skip the profiled iteration after the timed region (per-kernel breakdown)")
    p.add_argument("--gru-persist", type=int, default=3, choices=(0, 1, 2, 3),
                   help="recurrent: persistent whole-sequence GRU launches, bit 0 forward, bit 1 backward (3) or per-step launches (0)")
    p.add_argument("--products", type=int, default=6, choices=(6, 9),
                   help="part products per fp32 product in the split-bf16 GEMMs (9 = every product exact)")
    p.add_argument("--half-precision", action="store_true",
                   help="T/run.py --half-precision: Policy.half() (one bf16 MFMA product per GEMM product, fp32 "
                        "accumulation and masters) — a separate line, never the fp32 headline")
    p.add_argument("--tune", default="", help="key=v[,key=v...] ppo_tune_set overrides (A/B runs)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-envs", type=int, default=128)
    p.add_argument("--cpu-steps", type=int, default=32,
                   help="rollout steps per CPU-baseline iteration (per-env-step cost is independent of T)")
    p.add_argument("--cpu-reps", type=int, default=5)
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="threads of the multi-threaded CPU baseline (default: OMP_NUM_THREADS or the core count, <= 16)")
    p.add_argument("--no-gae-roofline", action="store_true")
    p.add_argument("--no-boundary", action="store_true", help="skip the observation-boundary measurement")
    p.add_argument("--gae-lanes", type=int, default=1 << 20)
    p.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                   help="collectives backend for N > 1 (nccl = RCCL; gloo only to rehearse on one GPU)")
    p.add_argument("--obs", default="u8", choices=("u8", "f32", "rgb"),
                   help="observation form: u8 4x84x84 synthetic frames (default, the headline); f32 = the reference's "
                        "fp32 storage plane fed by the f1/f2 chain (raw RGB frame -> NormalizeWrapper + "
                        "FrameStackMono(2) on the GPU, ppo_obs_preprocess); rgb = raw u8 RGB frames stored, the same "
                        "decode fused into conv1")
    p.add_argument("--force-collectives", action="store_true",
                   help="run every collective (parameter broadcast, advantage statistics, per-minibatch gradient "
                        "all-reduce, losses) even at N = 1, on a one-rank communicator of --dist-backend")
    return p.parse_args()


def gae_roofline(device, lanes, T=128, reps=10):
    """Fused GAE + advantage difference + moment partials on [T, lanes] planes.
    Algorithmic bytes per (t, lane): read r, v_t, m_{t+1} (12 B) + write ret, adv (8 B)."""
    from a2c_ppo_acktr._hip import call, stream
    g = torch.Generator(device=device).manual_seed(0)
    r = torch.rand(T, lanes, device=device, generator=g)
    v = torch.randn(T + 1, lanes, device=device, generator=g)
    m = (torch.rand(T + 1, lanes, device=device, generator=g) > 0.01).float()
    nv = torch.randn(lanes, device=device, generator=g)
    ret = torch.empty(T + 1, lanes, device=device)
    adv = torch.empty(T, lanes, device=device)
    parts = torch.empty(3 * call("ppo_gae_partials_count", lanes), dtype=torch.float64, device=device)
    s = stream()
    args = (r.data_ptr(), v.data_ptr(), m.data_ptr(), m.data_ptr(), nv.data_ptr(), ret.data_ptr(), adv.data_ptr(),
            parts.data_ptr(), T, lanes, 0.99, 0.95, 1, 0, s)
    call("ppo_compute_returns", *args)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call("ppo_compute_returns", *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = 20.0 * T * lanes
    gbps = nbytes / (ms * 1e-3) / 1e9
    del r, v, m, nv, ret, adv, parts
    torch.cuda.empty_cache()
    return {"bound": "hbm", "achieved": round(gbps, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": round(gbps / PEAK_HBM_GBPS, 4), "traffic": None,
            "config": f"T={T} x {lanes} lanes (fp32 planes, {nbytes / 1e9:.2f} GB algorithmic per launch)",
            "ms_per_launch": round(ms, 4), "small_shapes": gae_small(device)}


def gae_small(device, T=128, reps=50):
    """c1 / c2-sized compute_returns (8 and 1024 lanes): the bit-exact
    lane-sequential kernel (one thread per lane walks T steps) vs the
    time-parallel scan (16 lanes x 16 time chunks per block), µs per launch."""
    from a2c_ppo_acktr._hip import call, stream
    out = {}
    for lanes in (8, 1024, 4096):
        g = torch.Generator(device=device).manual_seed(1)
        r = torch.rand(T, lanes, device=device, generator=g)
        v = torch.randn(T + 1, lanes, device=device, generator=g)
        m = torch.ones(T + 1, lanes, device=device)
        nv = torch.randn(lanes, device=device, generator=g)
        ret = torch.empty(T + 1, lanes, device=device)
        adv = torch.empty(T, lanes, device=device)
        parts = torch.empty(2 * lanes, dtype=torch.float64, device=device)
        res = {}
        for name in ("ppo_compute_returns", "ppo_compute_returns_scan"):
            args = (r.data_ptr(), v.data_ptr(), m.data_ptr(), m.data_ptr(), nv.data_ptr(), ret.data_ptr(),
                    adv.data_ptr(), parts.data_ptr(), T, lanes, 0.99, 0.95, 1, 0, stream())
            call(name, *args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call(name, *args)
            e1.record()
            torch.cuda.synchronize()
            res["scan_us" if name.endswith("scan") else "exact_us"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
        out[f"{lanes}x{T}"] = res
    return out


def boundary_roofline(device, frames=16384, reps=5, cpu_frames=64):
    """Observation boundary: the fused NormalizeWrapper +
    FrameStackMono(2) + TransposeImage + .float() kernel on `frames` raw u8 RGB
    frames (algorithmic bytes per frame: 84*84*3 u8 in + 84*84*4 fp32 out), the
    pinned host->device rate of one rollout step of u8 frames (4096 envs), and
    the oracle's numpy restatement of the reference's per-env chain on the host."""
    from a2c_ppo_acktr.vec_env import ObsPreprocess
    S = 84
    g = torch.Generator(device=device).manual_seed(0)
    fr = torch.randint(0, 256, (frames, S, S, 3), dtype=torch.uint8, device=device, generator=g)
    mean = np.random.default_rng(0).uniform(20, 80, (S, S, 3))
    pre = ObsPreprocess(S, "norm", mean, 36.3, device=device)
    out = torch.empty(frames, 4, S, S, device=device)
    pre(fr, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pre(fr, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    per = S * S * (3 + 16)
    gbps = frames * per / (ms * 1e-3) / 1e9
    del fr, out
    host = torch.randint(0, 256, (4096, S, S, 3), dtype=torch.uint8).pin_memory()
    dev = torch.empty_like(host, device=device)
    dev.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        dev.copy_(host, non_blocking=True)
    e1.record()
    torch.cuda.synchronize()
    h2d_ms = e0.elapsed_time(e1) / reps
    del host, dev
    torch.cuda.empty_cache()
    from oracle import obs_oracle as OO
    cf = np.random.default_rng(1).integers(0, 256, (cpu_frames, S, S, 3), dtype=np.uint8)
    t0 = time.perf_counter()
    OO.preprocess_batch(cf, mean=mean, std=36.3)
    cpu_s = time.perf_counter() - t0
    return {"bound": "hbm", "achieved": round(gbps, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": round(gbps / PEAK_HBM_GBPS, 4), "kernel": "obs_preprocess (norm + grey + transpose + fp32)",
            "config": f"{frames} raw 84x84x3 u8 frames, {per} B algorithmic per frame",
            "frames_per_s": round(frames / (ms * 1e-3), 1), "ms_per_launch": round(ms, 4),
            "h2d_u8_step_ms": round(h2d_ms, 4),
            "h2d_u8_env_steps_per_s": round(4096 / (h2d_ms * 1e-3), 1),
            "cpu_baseline": {"value": round(cpu_frames / cpu_s, 1), "unit": "frames/s", "cores": 1, "kind": "port",
                             "sample": f"oracle numpy restatement of NormalizeWrapper + FrameStackMono(2) + "
                                       f"TransposeImage + .float() (013 chain), {cpu_frames} frames"}}


def eval_latency(device, H=256, V=14, steps=200, cpu_steps=20):
    """Evaluation path (SURVEY §8f f4, T/run_evaluation.py:25-122): one env,
    deterministic act with the GRU (H=256) + 14 vector obs of the OTC policy.
    Wall time per act, eager vs replayed from a HIP graph, synchronised each step
    (as the env loop needs the action), next to the oracle's float64 forward of
    one sample on the host."""
    from a2c_ppo_acktr.evaluation import GraphedActor
    from a2c_ppo_acktr.model import CNNBase, Policy
    from a2c_ppo_acktr.synthetic import Discrete
    torch.manual_seed(1)
    pol = Policy((4, 84, 84), Discrete(8), base=CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
                 vector_obs_len=V)
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy().astype(np.float64)
    pol.to(device)
    obs = torch.rand(1, 4, 84, 84, device=device)
    vec = torch.rand(1, V, device=device)
    hx = torch.zeros(1, H, device=device)
    m = torch.ones(1, 1, device=device)
    ga = GraphedActor(pol)
    gr = GraphedActor(pol, carry_hidden=True)   # the eval loop's form: inputs written in place, h fed back in-graph
    gr.obs.copy_(obs)
    gr.vec.copy_(vec)
    res = {}
    for name, fn in (("eager", lambda h: pol.act(obs, vec, h, m, deterministic=True)),
                     ("graph", lambda h: ga.act(obs, vec, h, m)),
                     ("replay", lambda h: gr.replay())):
        h = hx
        for _ in range(10):
            h = fn(h)[3]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            with torch.no_grad():
                _, a, _, h = fn(h)
            a.item()   # the env step needs the action on the host
        res[name] = (time.perf_counter() - t0) / steps * 1e3
    from oracle import ppo_oracle as O
    p = O.unflatten(flat, O.cnn_param_shapes(H, recurrent=True, vector_obs_len=V))
    o, v, h0 = np.random.rand(1, 4, 84, 84), np.random.rand(1, V), np.zeros((1, H))
    t0 = time.perf_counter()
    for _ in range(cpu_steps):
        O.recurrent_forward(p, o, v, h0, np.ones((1, 1)))
    cpu_ms = (time.perf_counter() - t0) / cpu_steps * 1e3
    return {"config": f"1 env, CNNBase+GRU H={H} + {V} vector obs, deterministic act, synchronised per step",
            "eager_ms_per_act": round(res["eager"], 4), "graph_ms_per_act": round(res["graph"], 4),
            "replay_ms_per_act": round(res["replay"], 4), "replay_acts_per_s": round(1e3 / res["replay"], 1),
            "note": "graph = GraphedActor.act (Policy.act signature: validity checks + input copies per act); "
                    "replay = GraphedActor.replay (inputs written in place, hidden state carried in-graph)",
            "cpu_baseline": {"value": round(cpu_ms, 3), "unit": "ms/act", "cores": 1, "kind": "port",
                             "sample": f"oracle float64 numpy forward of one sample, {cpu_steps} acts"}}


def pmc_traffic(kernel, workload):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC passes
    (profiles/roofline_traffic.json, written by tools/pmc_traffic.py) — only when
    they were measured on this same kernel and workload."""
    path = os.path.join(ROOT, "profiles", "roofline_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if d.get("kernel") != kernel or d.get("workload") != workload:
        return None, None
    return d.get("traffic_bytes_per_launch"), f"profiles/{d.get('tag', '?')}_traffic.json"


# bench kernel name -> the kernel symbol in the rocprofv3 PMC summaries
PMC_SYMBOL = {"conv2_fwd": ("conv2_fwd_x9c_kernel<", "conv2_fwd_lone_kernel<"),
              "conv2_dgrad": "conv2_dgrad_x9_kernel<", "conv2_wgrad": "conv2_wgrad_x9_kernel<",
              "conv3_fwd": ("conv3_fwd_c3_kernel<", "conv3_fwd_lone_kernel<", "conv3_fwd_x9_kernel<"),
              "conv3_dgrad": "conv3_dgrad_x9_kernel<", "conv3_wgrad": "conv3_wgrad_x9_kernel<",
              "trunk_fwd": "trunk_fwd_kernel<",
              "conv1_wgrad_u8": ("conv1_wgrad_kw3_kernel<", "conv1_wgrad_kw2_kernel<", "conv1_wgrad_parts_kernel<"),
              "conv1_fwd_u8": "conv1_fwd_bf16x3_kernel<"}


def pmc_mfma(workload):
    """Measured MFMA pipeline utilisation per bench kernel (SQ_VALU_MFMA_BUSY_CYCLES
    over SIMD-cycles, tools/profile_round.sh 'mfma' pass) — same workload only."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "roofline_traffic.json")))
        m = json.load(open(os.path.join(ROOT, d["mfma_util_file"])))
    except (OSError, ValueError, KeyError):
        return {}, {}, None
    if m.get("workload") != workload:
        return {}, {}, None
    out, clk = {}, {}
    for name, sym in PMC_SYMBOL.items():
        # all instantiations (e.g. the rollout and the mask-writing training
        # forward): busy cycles are proportional to MFMA instructions, so the
        # combined utilisation is Σ insts / Σ (insts / util)
        parts = [(v["mfma_insts_per_launch"] * v["launches"], v["mfma_util"])
                 for k, v in m["kernels"].items() if k.startswith(sym) and v["mfma_util"] > 0]
        if parts:
            out[name] = round(sum(w for w, _ in parts) / sum(w / u for w, u in parts), 4)
        # shader clock of the kernel's launches (cycles-weighted over its instantiations)
        cyc = [(v["sclk_ghz"] * v["pmc_avg_launch_ms"] * v["launches"], v["pmc_avg_launch_ms"] * v["launches"])
               for k, v in m["kernels"].items() if k.startswith(sym) and v.get("sclk_ghz")]
        if cyc:
            clk[name] = round(sum(c for c, _ in cyc) / sum(t for _, t in cyc), 4)
    return out, clk, d["mfma_util_file"]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(envs, T, E, M, hidden, threads, reps=3):
    """The reference's CPU path (T/run.py:168-248: act -> env -> insert x T,
    get_value, compute_returns, PPO.update with torch.optim.Adam and
    clip_grad_norm_, after_update) restated in torch (oracle/torch_ref.py, pinned
    to the reference's recorded iteration), fp32 observations as the reference
    stores them, `envs` lanes x T steps per iteration — at 1 thread (the
    reference's torch.set_num_threads(1), T/run.py:55) and at `threads`: a short
    warm-up iteration, then the median of `reps` timed iterations."""
    from a2c_ppo_acktr.model import CNNBase, Policy
    from a2c_ppo_acktr.synthetic import Discrete
    from oracle import torch_ref as TR
    saved = torch.get_num_threads()
    rng_state = torch.get_rng_state()
    torch.manual_seed(1)
    pol = Policy((4, 84, 84), Discrete(8), base=CNNBase, base_kwargs={"recurrent": False, "hidden_size": hidden})
    flat = torch.cat([q.detach().reshape(-1) for q in pol.parameters()])
    runs = {}
    try:
        for th in sorted({1, threads}):
            torch.set_num_threads(th)
            p = TR.unflatten(flat, hidden, requires_grad=True)
            opt = torch.optim.Adam(p, lr=1e-4, eps=1e-5)
            gen = torch.Generator().manual_seed(123)
            frames = TR.env_frames(envs, gen=gen)
            # one short warm-up iteration (allocator, thread pool), then the median of
            # `reps` whole iterations
            TR.run_iteration(p, opt, envs, max(T // 8, 1), ppo_epoch=1, num_mini_batch=M, gen=gen, frames=frames)
            times = []
            for _ in range(reps):
                t0 = time.perf_counter()
                TR.run_iteration(p, opt, envs, T, ppo_epoch=E, num_mini_batch=M, gen=gen, frames=frames)
                times.append(time.perf_counter() - t0)
            dt = sorted(times)[len(times) // 2]
            runs[th] = (envs * T / dt, dt, times)
    finally:
        torch.set_num_threads(saved)
        torch.set_rng_state(rng_state)
    best = max(runs, key=lambda k: runs[k][0])
    bt = runs[best][2]
    return {"value": round(runs[best][0], 2), "unit": "env-steps/s", "cores": best, "kind": "port",
            "cpu_model": cpu_model(),
            "runs_s": [round(x, 3) for x in bt],
            "range": [round(envs * T / max(bt), 2), round(envs * T / min(bt), 2)],
            "by_threads": {str(k): {"value": round(v[0], 2), "seconds": round(v[1], 2),
                                    "runs_s": [round(x, 3) for x in v[2]]} for k, v in runs.items()},
            "sample": f"the reference CPU path (T/run.py:168-248) restated in torch on the host "
                      f"(oracle/torch_ref.py: F.conv2d/linear, autograd, torch.optim.Adam, clip_grad_norm_, "
                      f"fp32 obs storage), CNNBase H={hidden}, {envs} envs x {T} steps, {E} epochs x {M} "
                      f"minibatches; per thread setting one warm-up iteration then the median of {reps} "
                      f"iterations (range = slowest..fastest of them); value = the faster setting"}


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks of this script as child
    processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each), wait
    for all of them, and return the first non-zero exit status.  Nothing here
    touches the GPU; if one rank fails the others are stopped (they would block
    in a collective)."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.kill()
        time.sleep(0.2)
    return rc


def kernel_entry(name, launches, ms_total, work, products, where):
    bound, peak, unit_kind, how = profiled(products).get(
        name, ("mfma", PEAK_FP32_MFMA_TFLOPS, "flop", "v_mfma_f32_32x32x2_f32"))
    if unit_kind == "bytes":
        achieved, unit = work / (ms_total * 1e-3) / 1e9, "GB/s"
    elif unit_kind == "conv1_flop":
        achieved, unit = work * CONV1_FWD_BYTES_PER_FLOP / (ms_total * 1e-3) / 1e9, "GB/s"
    else:
        achieved, unit = work / (ms_total * 1e-3) / 1e12, "TFLOP/s"
    e = {"bound": bound, "achieved": round(achieved, 2), "peak": round(peak, 1), "unit": unit,
         "frac": round(achieved / peak, 4), "ms_total": round(ms_total, 3), "launches": int(launches),
         "avg_launch_ms": round(ms_total / launches, 4), "instructions": how, "timed_in": where}
    if unit_kind != "bytes":
        e["fp32_tflops"] = round(work / (ms_total * 1e-3) / 1e12, 2)
    if name in CONV_HBM:   # the same launches against HBM: compulsory bytes per image
        macs, nbytes = CONV_HBM[name]
        gbps = work / (2.0 * macs) * nbytes / (ms_total * 1e-3) / 1e9
        e["hbm_view"] = {"bytes_per_image": nbytes, "achieved_gbps": round(gbps, 1),
                         "frac_of_hbm_peak": round(gbps / PEAK_HBM_GBPS, 4)}
    return e


def prof_collect(names):
    out = {}
    from a2c_ppo_acktr import _hip
    for ki, name in enumerate(names):
        prof = torch.zeros(3, dtype=torch.float64)
        _hip.call("ppo_prof_collect_one", ki, prof.data_ptr())
        out[name] = prof.tolist()
    _hip.call("ppo_prof_enable", None, 0)
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: one child process per rank (started before any GPU call here)
        if args.dist_backend == "nccl" and torch.cuda.device_count() < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but {torch.cuda.device_count()} GPUs are visible", file=sys.stderr)
            sys.exit(2)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} does not match --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; modulo the visible count only so a gloo rehearsal of the
    # N > 1 path can run several ranks on a one-GPU box (--dist-backend gloo)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world == 1 and args.force_collectives:   # a one-rank communicator, no launcher
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if world > 1 or args.force_collectives:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)   # RCCL over xGMI
        else:
            dist.init_process_group(args.dist_backend)
        assert dist.get_world_size() == args.gpus
    from a2c_ppo_acktr import _dist
    _dist.force_collectives(args.force_collectives)
    collectives = _dist.active()

    from a2c_ppo_acktr import _hip
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.model import CNNBase, Policy
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv

    _hip.call("ppo_tune_set", b"products", args.products)
    tune = {}
    for kv in [x for x in args.tune.split(",") if x]:
        k, v = kv.split("=")
        _hip.call("ppo_tune_set", k.encode(), int(v))
        tune[k] = int(v)
    _hip.call("ppo_gru_persist_set", args.gru_persist)
    N, T, E, M = args.envs, args.num_steps, args.ppo_epoch, args.num_mini_batch
    H = args.hidden or (256 if args.recurrent else 512)
    V = args.vec_len if args.recurrent else 0
    torch.manual_seed(1)
    frame_shape = (4, 84, 84) if args.obs == "u8" else (84, 84, 3)   # f32 / rgb: raw RGB frames from the env
    env = SyntheticVecEnv(N, obs_shape=frame_shape, seed=123 + 7919 * rank, p_done=0.01, device=device)
    policy = Policy((4, 84, 84), env.action_space, base=CNNBase,
                    base_kwargs={"recurrent": args.recurrent, "hidden_size": H}, vector_obs_len=V)
    policy.to(device)
    if args.half_precision:
        policy.half()
    pre = None
    if args.obs != "u8":
        from a2c_ppo_acktr.vec_env import ObsPreprocess
        # NormalizeWrapper("ObtRetro-v6")'s shapes: a fp32-valued mean [84][84][3] (synthetic: the reference's
        # file stays on the host) and its std value
        mean = np.random.default_rng(0).uniform(20, 80, (84, 84, 3)).astype(np.float32).astype(np.float64)
        pre = ObsPreprocess(84, "norm", mean, 36.31282043457031, mono=True, device=device)
        if args.obs == "rgb":
            policy.set_obs_decode(pre)
    agent = PPO(policy, 0.1, E, M, 0.5, 0.001, lr=1e-4, eps=1e-5, max_grad_norm=0.5)
    store_shape, store_dtype = {"u8": ((4, 84, 84), torch.uint8), "f32": ((4, 84, 84), torch.float32),
                                "rgb": ((84, 84, 3), torch.uint8)}[args.obs]
    rollouts = RolloutStorage(T, N, store_shape, [V], env.action_space, policy.recurrent_hidden_state_size,
                              obs_dtype=store_dtype, device=device)
    raw = torch.empty(N, 84, 84, 3, dtype=torch.uint8, device=device) if args.obs == "f32" else None

    def env_write(slot, action=None):
        """the env step into storage slot `slot`: f32 runs the f2 chain (raw frame ->
        fp32 4-channel policy input) as the reference's VecPyTorch feed does"""
        if raw is None:
            return env.step_into(slot, action) if action is not None else env.reset_into(slot)
        out = env.step_into(raw, action) if action is not None else env.reset_into(raw)
        pre(raw, out=slot)
        return out

    env_write(rollouts.obs[0])
    vec_src = torch.rand(N, V, device=device) if V else None   # synthetic vector obs (fixed)

    def iteration():
        for step in range(T):
            with torch.no_grad():
                value, action, logp, hxs = policy.act(rollouts.obs[step], rollouts.vector_obs[step],
                                                      rollouts.recurrent_hidden_states[step], rollouts.masks[step])
            slot = rollouts.obs[step + 1]
            reward, masks, bad_masks = env_write(slot, action)
            rollouts.insert(slot, vec_src if V else rollouts.vector_obs[step + 1], hxs, action, logp, value, reward,
                            masks, bad_masks)
        with torch.no_grad():
            next_value = policy.get_value(rollouts.obs[-1], rollouts.vector_obs[-1],
                                          rollouts.recurrent_hidden_states[-1], rollouts.masks[-1])
        rollouts.compute_returns(next_value, True, 0.99, 0.95, False)
        losses = agent.update(rollouts)
        rollouts.after_update()
        return losses

    for _ in range(args.warmup):
        iteration()
    torch.cuda.synchronize()

    gae = None
    if rank == 0 and not args.no_gae_roofline:
        gae = gae_roofline(device, args.gae_lanes)
    boundary = None
    if rank == 0 and not args.no_boundary:
        boundary = boundary_roofline(device)
    evalp = None
    if rank == 0 and not args.no_boundary:
        evalp = eval_latency(device)

    launches_per_iter = 8 * T + 32 * E * M + 64
    names = [k for k in args.profile_kernels.split(",") if k]
    _hip.call("ppo_prof_enable", ",".join(names).encode(), args.steps * launches_per_iter)
    _dist.time_grads(collectives)
    if collectives:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = None
    for _ in range(args.steps):
        losses = iteration()
    torch.cuda.synchronize()
    if collectives:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_kernel = prof_collect(names)
    _dist.time_grads(False)
    allreduce = None
    ar = _dist.grad_allreduce_times()
    if ar:
        # two buckets per minibatch for the CNN engines (_dist.start_bucket): the fc + heads
        # tail on a side stream, overlapped with the conv backward, and the conv head on
        # the engine's stream (exposed); one all-reduce of the whole buffer otherwise
        buckets = {}
        for t, nb in ar:
            b = buckets.setdefault(nb, [0.0, 0])
            b[0] += t
            b[1] += 1
        ms = sum(t for t, _ in ar)
        nbytes = sum(buckets)
        per_mb = max(b[1] for b in buckets.values())
        allreduce = {"backend": "rccl" if args.dist_backend == "nccl" else args.dist_backend, "world": world,
                     "per_minibatch_ms": round(ms / per_mb, 4), "launches": len(ar), "bytes": nbytes,
                     "ms_per_iteration": round(ms / args.steps, 3),
                     "algbw_GBps": round(nbytes / (ms / per_mb * 1e-3) / 1e9, 1),
                     "buckets": [{"bytes": nb, "per_minibatch_ms": round(b[0] / b[1], 4),
                                  "stream": "side (overlapped)" if nb == max(buckets) and len(buckets) > 1
                                  else "engine"} for nb, b in sorted(buckets.items(), reverse=True)],
                     "note": "HIP events around each gradient all-reduce inside the timed region, on the stream "
                             "it runs on (the fc + heads bucket on a side stream during the conv backward)"}

    # per-kernel breakdown: one more iteration with every kernel family event-timed
    # (outside the timed region: the extra events would perturb `value`)
    pass_info, pass_kernels = None, {}
    if not args.no_profile_pass:
        all_names = list(profiled(args.products))
        _hip.call("ppo_prof_enable", ",".join(all_names).encode(), launches_per_iter * 2)
        torch.cuda.synchronize()
        tp = time.perf_counter()
        iteration()
        torch.cuda.synchronize()
        pass_ms = (time.perf_counter() - tp) * 1e3
        pass_kernels = prof_collect(all_names)
        covered = sum(v[1] for v in pass_kernels.values())
        pass_info = {"iteration_ms": round(pass_ms, 2), "event_timed_ms": round(covered, 2),
                     "coverage": round(covered / pass_ms, 4),
                     "note": "sum of the event-timed kernel families / wall time of one profiled iteration"}

    if collectives:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if rank != 0:
        dist.destroy_process_group()
        return

    obs_desc = {"u8": "", "f32": ", fp32 obs storage fed by the f2 chain (--obs f32)",
                "rgb": ", raw RGB obs storage, decode fused into conv1 (--obs rgb)"}[args.obs]
    workload = ((f"c5: CNNBase+GRU H={H} + {V} vector obs" if args.recurrent else f"c3: CNNBase H={H}")
                + obs_desc + f", {N} env lanes x {T} steps per GPU, PPO {E} epochs x {M} minibatches "
                  f"(rollout + GAE + update, " + ("--half-precision: bf16 GEMM operands, fp32 accumulation"
                                                  if args.half_precision else "fp32") + ")")
    kernels = {}
    products = 1 if args.half_precision else args.products
    for name, (launches, ms_total, work) in per_kernel.items():
        if launches > 0 and ms_total > 0:
            kernels[name] = kernel_entry(name, launches, ms_total, work, products, "timed region")
    for name, (launches, ms_total, work) in pass_kernels.items():
        if launches > 0 and ms_total > 0:
            e = kernel_entry(name, launches, ms_total, work, products, "profile pass")
            e["ms_per_iteration"] = round(ms_total, 3)
            if name in kernels:
                kernels[name]["ms_per_iteration"] = e["ms_per_iteration"]
            else:
                kernels[name] = e
    util, clk, util_src = pmc_mfma(workload)
    for name, u in util.items():
        if name in kernels:
            kernels[name]["mfma_util_pmc"] = u
    for name, c in clk.items():
        # frac is against the nominal 2.4 GHz peak (the headline); frac_at_clock
        # against the peak at the clock the kernel was measured at in the PMC pass
        if name in kernels:
            kernels[name]["sclk_ghz_pmc"] = c
            kernels[name]["frac_at_clock"] = round(kernels[name]["frac"] * NOMINAL_SCLK_GHZ / c, 4)
    roof = None
    timed = {k: v for k, v in kernels.items() if v["timed_in"] == "timed region"}
    if timed:
        dom = max(timed, key=lambda k: timed[k]["ms_total"])
        kd = kernels[dom]
        traffic, tsrc = pmc_traffic(dom, workload)
        roof = {"bound": kd["bound"], "achieved": kd["achieved"], "peak": kd["peak"], "unit": kd["unit"],
                "frac": kd["frac"], "traffic": round(traffic) if traffic else None,
                "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": tsrc, "kernel": dom,
                "launches": kd["launches"], "avg_launch_ms": kd["avg_launch_ms"],
                "mfma_util_pmc": kd.get("mfma_util_pmc"), "mfma_util_source": util_src,
                "sclk_ghz_pmc": kd.get("sclk_ghz_pmc"), "frac_at_clock": kd.get("frac_at_clock"),
                "flop_per_launch": round(per_kernel[dom][2] / per_kernel[dom][0])}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1))
        cpu = cpu_baseline(args.cpu_envs, args.cpu_steps, E, M, H, threads, reps=args.cpu_reps)
    value = N * T * world * args.steps / elapsed
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if args.half_precision else "f32",
        "split_products": 1 if args.half_precision else args.products,
        "tune": tune or None,
        "data": ("synthetic: counter-hash u8 4x84x84 obs" if args.obs == "u8" else
                 "synthetic: counter-hash u8 84x84x3 RGB frames, NormalizeWrapper(synthetic fp32 mean, std 36.31) + "
                 "FrameStackMono(2)") + ", U[0,1) rewards, Bernoulli(0.01) dones; random-init weights",
        "config": {"workload": workload,
                   "envs_per_gpu": N, "num_steps": T, "ppo_epoch": E, "num_mini_batch": M, "hidden": H,
                   "obs": args.obs,
                   "global_batch": N * T * world, "parallelism": f"dp{world}",
                   "dist_backend": (args.dist_backend if collectives else None),
                   "collectives": ("forced at N=1" if collectives and world == 1 else
                                   "per minibatch" if collectives else "none (N=1)")},
        "allreduce": allreduce,
        "roofline": roof, "cpu_baseline": cpu, "gae_roofline": gae, "boundary_roofline": boundary, "eval_latency": evalp,
        "profile_pass": pass_info, "kernel_rooflines": kernels,
        "losses": [round(x, 6) for x in losses],
    }
    print(json.dumps(out), flush=True)
    if collectives:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
