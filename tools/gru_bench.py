#!/usr/bin/env python3
"""Times the whole-sequence GRU launches at the c5 minibatch (T = 256 steps x
n = 512 env columns, H = 256) through the C ABI for each ppo_gru_persist mode:
  python tools/gru_bench.py [--modes 0,1,5] [--reps 5]
bit 0: persistent forward (bit 2: hand-off in tagged data), bit 1: persistent BPTT."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import torch  # noqa: E402

from a2c_ppo_acktr._hip import call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="0,1,5")
    a = ap.parse_args()
    T, n, H = a.T, a.n, a.H
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    R = T * n
    h0 = torch.randn(n, H, device=dev, generator=g)
    whh = torch.randn(3 * H, H, device=dev, generator=g) / H ** 0.5
    whhT = whh.t().contiguous()
    bhh = torch.randn(3 * H, device=dev, generator=g) * 0.1
    gi = torch.randn(R, 3 * H, device=dev, generator=g)
    masks = (torch.rand(R, device=dev, generator=g) > 0.01).float()
    o = {k: torch.empty(R, H, device=dev) for k in ("h", "r", "z", "n", "ghn", "hin")}
    dout = torch.randn(R, H, device=dev, generator=g) * 1e-2
    dgi = torch.empty(R, 3 * H, device=dev)
    dgh = torch.empty(R, 3 * H, device=dev)
    dhz = torch.zeros(n, H, device=dev)
    carry = torch.zeros(n, H, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    prev = call("ppo_gru_persist_get")

    def fwd():
        call("ppo_gru_seq_fwd", h0.data_ptr(), masks.data_ptr(), None, whh.data_ptr(), bhh.data_ptr(), gi.data_ptr(),
             T, n, H, o["h"].data_ptr(), o["r"].data_ptr(), o["z"].data_ptr(), o["n"].data_ptr(), o["ghn"].data_ptr(),
             o["hin"].data_ptr(), s)

    def bwd():
        call("ppo_gru_seq_bwd", dout.data_ptr(), o["r"].data_ptr(), o["z"].data_ptr(), o["n"].data_ptr(),
             o["ghn"].data_ptr(), o["hin"].data_ptr(), masks.data_ptr(), None, whhT.data_ptr(), T, n, H,
             dgi.data_ptr(), dgh.data_ptr(), dhz.data_ptr(), carry.data_ptr(), s)

    ref = None
    try:
        for m in [int(x) for x in a.modes.split(",")]:
            call("ppo_gru_persist_set", m)
            for name, fn in (("fwd", fwd), ("bwd", bwd)):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                print(f"mode {m} {name}: {ms:7.3f} ms  {1e3 * ms / T:6.2f} us/step", flush=True)
            if ref is None:
                ref = o["h"].clone()
            else:
                print(f"mode {m} hout bit-identical to mode {a.modes.split(',')[0]}: {torch.equal(ref, o['h'])}")
            assert call("ppo_gru_persist_timeouts", s) == 0
    finally:
        call("ppo_gru_persist_set", prev)


if __name__ == "__main__":
    main()
