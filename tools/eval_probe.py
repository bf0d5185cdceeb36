#!/usr/bin/env python3
"""Batch-1 evaluation act (GraphedActor and eager), for a rocprofv3 kernel-trace
of the per-kernel latency chain (bench.py eval_latency's workload)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]
import torch  # noqa: E402

from a2c_ppo_acktr.evaluation import GraphedActor  # noqa: E402
from a2c_ppo_acktr.model import CNNBase, Policy  # noqa: E402
from a2c_ppo_acktr.synthetic import Discrete  # noqa: E402

dev = torch.device("cuda:0")
H, V = 256, 14
torch.manual_seed(1)
pol = Policy((4, 84, 84), Discrete(8), base=CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
             vector_obs_len=V)
pol.to(dev)
u8 = "--u8" in sys.argv
obs = (torch.randint(0, 256, (1, 4, 84, 84), dtype=torch.uint8, device=dev) if u8
       else torch.rand(1, 4, 84, 84, device=dev))
vec, h, m = torch.rand(1, V, device=dev), torch.zeros(1, H, device=dev), torch.ones(1, 1, device=dev)
ga = GraphedActor(pol)
for name, fn in (("eager", lambda h: pol.act(obs, vec, h, m, deterministic=True)), ("graph", lambda h: ga.act(obs, vec, h, m))):
    for _ in range(10):
        h = fn(h)[3]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        with torch.no_grad():
            _, a, _, h = fn(h)
        a.item()
    print(name, (time.perf_counter() - t0) * 10, "ms per act", flush=True)
ga2 = GraphedActor(pol, carry_hidden=True)
ga2.obs.copy_(obs)
ga2.vec.copy_(vec)
for _ in range(10):
    ga2.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100):
    out = ga2.replay()
    out[1].item()
print("replay", (time.perf_counter() - t0) * 10, "ms per act", flush=True)
