#!/usr/bin/env python3
"""CU contention between the persistent conv kernels (one 512-thread block per
CU holding 256 VGPRs per lane: the whole register file) and a kernel on a side
stream standing in for the gradient all-reduce's collective (DESIGN.md §7,
VERDICT r03 item 8; _dist.start_bucket overlaps the fc + heads bucket with the
conv backward).  The stand-in (ppo_probe_side_kernel) holds `--side-blocks`
workgroups for `--side-us` microseconds each and records when each started.

Printed per case: the conv kernel's time, the side kernel's time (both from one
common start event), and when the side blocks started relative to that event.
  python tools/cu_contention.py [--B 65536] [--side-blocks 256] [--side-us 200]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import torch  # noqa: E402

from a2c_ppo_acktr._hip import call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--side-blocks", type=int, default=256)
    ap.add_argument("--side-threads", type=int, default=256)
    ap.add_argument("--side-us", type=float, default=200.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B = a.B
    g = torch.Generator(device=dev).manual_seed(0)
    packed = torch.empty(call("ppo_packed_weights_size", 512), device=dev)
    offs = torch.zeros(6, dtype=torch.int64)
    call("ppo_packed_offsets", 512, offs.data_ptr())
    pk = [packed.data_ptr() + 4 * int(o) for o in offs]
    w2 = torch.randn(64, 512, device=dev, generator=g) * 0.05
    w3 = torch.randn(32, 576, device=dev, generator=g) * 0.05
    w4 = torch.randn(512, 1568, device=dev, generator=g) * 0.02
    main_s = torch.cuda.current_stream()
    s = main_s.cuda_stream
    call("ppo_pack_weights", w2.data_ptr(), w3.data_ptr(), w4.data_ptr(), 512, packed.data_ptr(), s)
    dz2 = torch.randn(B * 81 * 64, device=dev, generator=g)
    m1 = torch.randint(-2 ** 31, 2 ** 31 - 1, (B * 400,), dtype=torch.int32, device=dev, generator=g)
    dz1 = torch.empty(B * 400 * 32, device=dev)
    side = torch.cuda.Stream(dev)
    nb = a.side_blocks
    stamps = torch.zeros(nb * 2, dtype=torch.int64, device=dev)
    t0 = torch.zeros(1, dtype=torch.int64, device=dev)
    ticks = int(a.side_us * 100)   # 100 MHz counter

    def conv():
        call("ppo_conv2_dgrad_bits", dz2.data_ptr(), B, pk[5], m1.data_ptr(), dz1.data_ptr(), s)

    def side_k():
        call("ppo_probe_side_kernel", nb, a.side_threads, ticks, stamps.data_ptr(), side.cuda_stream)

    def run(order):
        ev0 = torch.cuda.Event(enable_timing=True)
        ec, es = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        call("ppo_probe_now", t0.data_ptr(), s)
        ev0.record(main_s)
        side.wait_event(ev0)
        if order == "conv_only":
            conv()
        elif order == "side_only":
            with torch.cuda.stream(side):
                side_k()
        elif order == "conv_then_side":
            conv()
            with torch.cuda.stream(side):
                side_k()
        else:   # side_then_conv
            with torch.cuda.stream(side):
                side_k()
            conv()
        ec.record(main_s)
        es.record(side)
        torch.cuda.synchronize()
        out = {"order": order}
        if order != "side_only":
            out["conv_ms"] = round(ev0.elapsed_time(ec), 4)
        if order != "conv_only":
            st = stamps.view(nb, 2).cpu()
            base = int(t0.item())
            starts = (st[:, 0] - base).double() / 100.0   # us
            out["side_ms"] = round(ev0.elapsed_time(es), 4)
            out["side_start_us"] = {"first": round(starts.min().item(), 1), "median": round(starts.median().item(), 1),
                                    "last": round(starts.max().item(), 1)}
        return out

    conv()
    torch.cuda.synchronize()
    res = []
    for _ in range(a.reps):
        for order in ("conv_only", "side_only", "conv_then_side", "side_then_conv"):
            res.append(run(order))
    for r in res:
        print(json.dumps(r), flush=True)
    summary = {}
    for order in ("conv_only", "side_only", "conv_then_side", "side_then_conv"):
        rs = [r for r in res if r["order"] == order]
        summary[order] = {k: round(sorted(r[k] for r in rs)[len(rs) // 2], 4) for k in ("conv_ms", "side_ms")
                          if k in rs[0]}
        if "side_start_us" in rs[0]:
            summary[order]["side_first_start_us"] = sorted(r["side_start_us"]["first"] for r in rs)[len(rs) // 2]
            summary[order]["side_last_start_us"] = sorted(r["side_start_us"]["last"] for r in rs)[len(rs) // 2]
    print(json.dumps({"cu_contention": summary, "B": B, "side_blocks": nb, "side_threads": a.side_threads,
                      "side_us": a.side_us, "conv_kernel": "conv2_dgrad_x9 (persistent, one block per CU)"}),
          flush=True)


if __name__ == "__main__":
    main()
