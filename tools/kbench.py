#!/usr/bin/env python3
"""Per-kernel micro-benchmark of the trunk GEMMs at the PPO minibatch size
(B = 4096*128/8 = 65536 samples) through the C ABI.  Prints ms and TFLOP/s per
kernel; used with rocprofv3 --pmc for counter passes.

  python tools/kbench.py [--B 65536] [--reps 5] [--only conv1_fwd,conv2_dgrad]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import torch  # noqa: E402

from a2c_ppo_acktr._hip import call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--tune", default="", help="key=v[,key=v...] tile variants (ppo_tune_set)")
    ap.add_argument("--z2", type=int, default=0, help="conv2 wgrad split count (default: ppo_wgrad_splits)")
    ap.add_argument("--z1", type=int, default=0, help="conv1 wgrad split count (default: ppo_wgrad_splits)")
    ap.add_argument("--z3", type=int, default=0, help="conv3 wgrad split count (default: ppo_wgrad_splits)")
    ap.add_argument("--z4", type=int, default=0, help="fc wgrad split count (default: ppo_wgrad_splits)")
    a = ap.parse_args()
    for kv in [x for x in a.tune.split(",") if x]:
        k, v = kv.split("=")
        call("ppo_tune_set", k.encode(), int(v))
    B, H = a.B, a.H
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    rows = B + 4096
    obs = torch.randint(0, 256, (rows, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    idx = torch.randperm(rows, device=dev)[:B].contiguous()

    def rn(*s, sc=0.05):
        return torch.randn(*s, device=dev, generator=g) * sc

    w1, b1 = rn(32, 256), rn(32)
    w2, b2 = rn(64, 512), rn(64)
    w3, b3 = rn(32, 576), rn(32)
    w4, b4 = rn(H, 1568), rn(H)
    packed = torch.empty(call("ppo_packed_weights_size", H), device=dev)
    offs = torch.zeros(6, dtype=torch.int64)
    call("ppo_packed_offsets", H, offs.data_ptr())
    pk = [packed.data_ptr() + 4 * int(o) for o in offs]
    s = torch.cuda.current_stream().cuda_stream
    call("ppo_pack_weights", w2.data_ptr(), w3.data_ptr(), w4.data_ptr(), H, packed.data_ptr(), s)
    a1 = torch.empty(B * 400 * 32, device=dev)
    m1 = torch.empty(B * 400, dtype=torch.int32, device=dev)   # ReLU mask bits of a1, a2
    m2 = torch.empty(B * 81, dtype=torch.int64, device=dev)
    m3 = torch.empty(B * 49, dtype=torch.int32, device=dev)
    a2 = torch.empty(B * 81 * 64, device=dev)
    a3 = torch.empty(B * 1568, device=dev)
    h = torch.empty(B * H, device=dev)
    dh = rn(B * H, sc=1e-3)
    dz3 = torch.empty(B * 1568, device=dev)
    dz2 = torch.empty(B * 81 * 64, device=dev)
    dz1 = torch.empty(B * 400 * 32, device=dev)
    gw = torch.empty(H * 1568 + 1024, device=dev)
    gb = torch.empty(1024, device=dev)
    Zmax = 4096
    slab = torch.empty(Zmax * 32 * 576 + Zmax * 64 * 512, device=dev)
    slab_b = torch.empty(Zmax * 512, device=dev)

    def zs(R, tiles):
        return call("ppo_wgrad_splits", R, tiles, 2048, 16)

    z1, z2, z3, z4 = zs(B * 400, 1), zs(B * 81, 4), zs(B * 49, 5), zs(B, ((H + 127) // 128) * 13)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    z1c = a.z1 or max(n_cu, -(-B // 512))   # the engine's split for the image-resident conv1 wgrads
    z2 = a.z2 or z2
    z1 = a.z1 or z1
    z3 = a.z3 or z3
    z4 = a.z4 or z4
    fws = torch.empty(max(call("ppo_fc_fwd_ws_bytes", B, H) // 4, 4), device=dev)
    z2c = a.z2 or max(n_cu, -(-B // 512))   # the engine's split for the image-resident conv2 wgrad
    gru = any(k.startswith("gru_") for k in a.only.split(","))
    gx, gwih, gbih = (rn(B * 272, sc=1.0), rn(768 * 272), rn(768)) if gru else (None, None, None)
    ggi = rn(B * 768, sc=1.0) if gru else None
    ghp, gho = (rn(B * 256, sc=0.5), torch.empty(B * 256, device=dev)) if gru else (None, None)
    gwhh, gbhh = (rn(768 * 256), rn(768)) if gru else (None, None)
    hw = rn(9 * H + 9, sc=0.03)                       # heads: wc [H], bc, wa [8][H], ba [8]
    hv = torch.empty(3 * B, device=dev)
    ha = torch.empty(B, dtype=torch.int64, device=dev)
    obs32 = frames = mean = None
    if any(k.endswith(("_f32", "_rgb")) for k in a.only.split(",")):
        obs32 = (torch.randn(rows, 4, 84, 84, device=dev, generator=g) * 0.8).contiguous()
        frames = torch.randint(0, 256, (rows, 84, 84, 3), dtype=torch.uint8, device=dev, generator=g)
        mean = torch.rand(84, 84, 3, device=dev, generator=g) * 60 + 20
    # heads_train inputs: storage planes indexed by idx (the minibatch rows), partials
    # sized for 32 rows per wave or fewer
    st_act = torch.randint(0, 8, (rows,), dtype=torch.int64, device=dev, generator=g)
    st_f = rn(4, rows, sc=1.0)   # old_logp, adv, vpred, ret
    st_f[0] = -st_f[0].abs() - 1.0
    hmax = -(-B // 32)
    part = torch.empty(hmax * (9 * H + 9 + 4), device=dev)

    def heads_train():
        nb = call("ppo_heads_train_blocks", B)
        call("ppo_heads_train", h.data_ptr(), None, B, H, hw.data_ptr(), hw.data_ptr() + 4 * H,
             hw.data_ptr() + 4 * (H + 1), hw.data_ptr() + 4 * (9 * H + 1), 8, idx.data_ptr(), 0, st_act.data_ptr(),
             st_f[0].data_ptr(), st_f[1].data_ptr(), st_f[2].data_ptr(), st_f[3].data_ptr(), 0.1, 0.5, 0.01, 1.0 / B, 1,
             1, dz3.data_ptr(), None, part.data_ptr(), part.data_ptr() + 4 * nb * 9 * H,
             part.data_ptr() + 4 * nb * (9 * H + 9), s)

    K = {
        "heads_train": (heads_train, 0.0),
        "conv1_fwd": (lambda: call("ppo_conv1_fwd", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(),
                                   b1.data_ptr(), a1.data_ptr(), s), 2.0 * B * 400 * 32 * 256),
        "conv2_fwd": (lambda: call("ppo_conv2_fwd", a1.data_ptr(), B, pk[0], b2.data_ptr(), a2.data_ptr(), s),
                      2.0 * B * 81 * 64 * 512),
        "conv3_fwd": (lambda: call("ppo_conv3_fwd", a2.data_ptr(), B, pk[1], b3.data_ptr(), a3.data_ptr(), s),
                      2.0 * B * 49 * 32 * 576),
        "fc_fwd": (lambda: call("ppo_fc_fwd", a3.data_ptr(), B, pk[2], b4.data_ptr(), H, h.data_ptr(), H, s),
                   2.0 * B * 1568 * H),
        "fc_fwd_ws": (lambda: call("ppo_fc_fwd_ws", a3.data_ptr(), B, pk[2], b4.data_ptr(), H, h.data_ptr(), H,
                                   fws.data_ptr(), fws.numel() * 4, s), 2.0 * B * 1568 * H),
        # the c5 GRU input projection x [B][272] . W_ih^T (768 x 272) + b (ppo_linear_fwd_ex)
        "gru_in": (lambda: call("ppo_linear_fwd_ex", a3.data_ptr(), None, B, 272, 272, w4.data_ptr(), None, 768,
                                dz3.data_ptr(), 768, 0, s), 2.0 * B * 768 * 272),   # dz3: B x 1568 >= B x 768
        # the rollout heads (Categorical sample, value, log-prob, entropy) on B rows of H features
        "heads_act": (lambda: call("ppo_heads_act", h.data_ptr(), None, B, H, hw.data_ptr(), hw.data_ptr() + 4 * H,
                                   hw.data_ptr() + 4 * (H + 1), hw.data_ptr() + 4 * (9 * H + 1), 8, None, 7, 0, 0,
                                   None, hv.data_ptr(), ha.data_ptr(), hv.data_ptr() + 4 * B, hv.data_ptr() + 8 * B,
                                   s), 0.0),
        # the c5 GRU input gradient dh = (dgi [B][768] . W_ih[:, :256]) masked by the fc ReLU (ppo_linear_dgrad_ex)
        "gru_dx": (lambda: call("ppo_linear_dgrad_ex", dz3.data_ptr(), B, 768, w4.data_ptr(), 256, a3.data_ptr(), 1568,
                                1, dz2.data_ptr(), s), 2.0 * B * 768 * 256),
        "fc_fwd_generic": (lambda: call("ppo_linear_relu_fwd", a3.data_ptr(), B, 1568, pk[2], b4.data_ptr(), H,
                                        h.data_ptr(), s), 2.0 * B * 1568 * H),
        "fc_dgrad": (lambda: call("ppo_linear_dgrad_mask", dh.data_ptr(), B, H, pk[3], 1568, a3.data_ptr(),
                                  dz3.data_ptr(), s), 2.0 * B * 1568 * H),
        "conv3_fwd_mask": (lambda: call("ppo_conv3_fwd_mask", a2.data_ptr(), B, pk[1], b3.data_ptr(), a3.data_ptr(),
                                        m3.data_ptr(), s), 2.0 * B * 49 * 32 * 576),
        "fc_dgrad_bits": (lambda: call("ppo_fc_dgrad_bits", dh.data_ptr(), B, H, pk[3], m3.data_ptr(), dz3.data_ptr(),
                                       s), 2.0 * B * 1568 * H),
        # the fc dgrad without the ReLU-mask read (bounds what mask bits could save)
        "fc_dgrad_nomask": (lambda: call("ppo_linear_dgrad_mask", dh.data_ptr(), B, H, pk[3], 1568, None,
                                         dz3.data_ptr(), s), 2.0 * B * 1568 * H),
        "fc_wgrad": (lambda: call("ppo_linear_wgrad", dh.data_ptr(), a3.data_ptr(), B, H, 1568, z4, slab.data_ptr(),
                                  slab_b.data_ptr(), s), 2.0 * B * 1568 * H),
        "fc_wreduce": (lambda: call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), z4, H, 1568, 2, 32, 49,
                                    gw.data_ptr(), gb.data_ptr(), 1.0, 0, s), 0.0),
        "conv3_dgrad": (lambda: call("ppo_conv3_dgrad", dz3.data_ptr(), B, pk[4], a2.data_ptr(), dz2.data_ptr(), s),
                        2.0 * B * 49 * 32 * 576),
        "conv3_wgrad": (lambda: call("ppo_conv3_wgrad", dz3.data_ptr(), a2.data_ptr(), B, z3, slab.data_ptr(),
                                     slab_b.data_ptr(), s), 2.0 * B * 49 * 32 * 576),
        "conv2_dgrad": (lambda: call("ppo_conv2_dgrad", dz2.data_ptr(), B, pk[5], a1.data_ptr(), dz1.data_ptr(), s),
                        2.0 * B * 81 * 64 * 512),
        # training-forward variants that also write ReLU mask bits, and the dgrads
        # that read the bits instead of the fp32 activations (the engine's path)
        "conv1_fwd_mask": (lambda: call("ppo_conv1_fwd_mask", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B,
                                        w1.data_ptr(), b1.data_ptr(), a1.data_ptr(), m1.data_ptr(), s),
                           2.0 * B * 400 * 32 * 256),
        "conv2_fwd_mask": (lambda: call("ppo_conv2_fwd_mask", a1.data_ptr(), B, pk[0], b2.data_ptr(), a2.data_ptr(),
                                        m2.data_ptr(), s), 2.0 * B * 81 * 64 * 512),
        "conv3_dgrad_bits": (lambda: call("ppo_conv3_dgrad_bits", dz3.data_ptr(), B, pk[4], m2.data_ptr(),
                                          dz2.data_ptr(), s), 2.0 * B * 49 * 32 * 576),
        "conv2_dgrad_bits": (lambda: call("ppo_conv2_dgrad_bits", dz2.data_ptr(), B, pk[5], m1.data_ptr(),
                                          dz1.data_ptr(), s), 2.0 * B * 81 * 64 * 512),
        "conv2_wgrad": (lambda: call("ppo_conv2_wgrad", dz2.data_ptr(), a1.data_ptr(), B, z2, slab.data_ptr(),
                                     slab_b.data_ptr(), s), 2.0 * B * 81 * 64 * 512),
        "conv1_wgrad": (lambda: call("ppo_conv1_wgrad", dz1.data_ptr(), obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, z1,
                                     slab.data_ptr(), slab_b.data_ptr(), s), 2.0 * B * 400 * 32 * 256),
        "conv1_fwd_f32": (lambda: call("ppo_conv1_fwd_f32", obs32.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(),
                                       b1.data_ptr(), a1.data_ptr(), m1.data_ptr(), s), 2.0 * B * 400 * 32 * 256),
        "conv1_fwd_rgb": (lambda: call("ppo_conv1_fwd_rgb", frames.data_ptr(), idx.data_ptr(), 0, B, mean.data_ptr(),
                                       36.31282043457031, w1.data_ptr(), b1.data_ptr(), a1.data_ptr(), m1.data_ptr(),
                                       s), 2.0 * B * 400 * 32 * 256),
        "conv1_wgrad_f32": (lambda: call("ppo_conv1_wgrad_f32", dz1.data_ptr(), obs32.data_ptr(), idx.data_ptr(), 0, B,
                                         z1c, slab.data_ptr(), slab_b.data_ptr(), s), 2.0 * B * 400 * 32 * 256),
        "conv1_wgrad_rgb": (lambda: call("ppo_conv1_wgrad_rgb", dz1.data_ptr(), frames.data_ptr(), idx.data_ptr(), 0,
                                         B, mean.data_ptr(), 36.31282043457031, z1c, slab.data_ptr(),
                                         slab_b.data_ptr(), s), 2.0 * B * 400 * 32 * 256),
        # the recurrent trunk's GRU input projection gi = x_pad · W_ihᵀ + b (c5: K = 272, N = 768)
        "gru_gi": (lambda: call("ppo_linear_fwd_ex", gx.data_ptr(), None, B, 272, 272, gwih.data_ptr(),
                                gbih.data_ptr(), 768, ggi.data_ptr(), 768, 0, s), 2.0 * B * 272 * 768),
        # the rollout's GRU step (c5: H = 256)
        "gru_step": (lambda: call("ppo_gru_step_fwd", ghp.data_ptr(), None, None, gwhh.data_ptr(), gbhh.data_ptr(),
                                  ggi.data_ptr(), B, 256, gho.data_ptr(), None, None, None, None, None, s),
                     2.0 * B * 768 * 256),
        "conv1_wreduce": (lambda: call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), z1, 32, 256, 0, 0, 0,
                                       gw.data_ptr(), gb.data_ptr(), 1.0 / 255, 0, s), 0.0),
        # the rollout's fused trunk (conv1 -> conv2 -> conv3 in one launch) on one rollout step's 4,096 images
        "trunk_4096": (lambda: call("ppo_trunk_fwd", obs.data_ptr(), idx.data_ptr(), 0, min(B, 4096), w1.data_ptr(),
                                    b1.data_ptr(), a1.data_ptr(), None, pk[0], b2.data_ptr(), a2.data_ptr(), None,
                                    pk[1], b3.data_ptr(), a3.data_ptr(), s),
                       2.0 * min(B, 4096) * (400 * 32 * 256 + 81 * 64 * 512 + 49 * 32 * 576)),
    }
    # realistic activations for the backward kernels
    K["conv1_fwd_mask"][0](); K["conv2_fwd_mask"][0](); K["conv3_fwd_mask"][0](); K["fc_fwd"][0]()
    K["fc_dgrad"][0](); K["conv3_dgrad"][0](); K["conv2_dgrad"][0]()
    torch.cuda.synchronize()
    # default: the c3 iteration's kernels (the engine's training forms) and the rollout trunk
    only = [x for x in a.only.split(",") if x] or [
        "conv1_fwd_mask", "conv2_fwd_mask", "conv3_fwd_mask", "fc_fwd", "fc_dgrad_bits", "fc_wgrad", "conv3_dgrad_bits",
        "conv3_wgrad", "conv2_dgrad_bits", "conv2_wgrad", "conv1_wgrad", "conv1_fwd", "conv2_fwd", "trunk_4096"]
    total = 0.0
    for name, (fn, fl) in K.items():
        if only and name not in only:
            continue
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        total += ms
        tf = fl / (ms * 1e-3) / 1e12 if fl else 0.0
        print(f"{name:14s} {ms:8.3f} ms  {tf:7.1f} TFLOP/s", flush=True)
    print(f"{'total':14s} {total:8.3f} ms")


if __name__ == "__main__":
    main()
