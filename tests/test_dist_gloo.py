"""The N>1 protocol (a2c_ppo_acktr/_dist.py) on CPU with gloo, world_size 2:
sharded lanes see the single-process advantage statistics, and the averaged
gradient drives an identical clip + Adam step on every rank."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_DIR, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    for p in (ROOT, PKG_DIR):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from a2c_ppo_acktr import _dist
    from oracle import ppo_oracle as O
    rng = np.random.default_rng(0)
    T, N = 16, 12                       # global lanes, split 6 + 6
    ret = (3 * rng.standard_normal((T + 1, N)) + 1).astype(np.float32)
    val = (3 * rng.standard_normal((T + 1, N))).astype(np.float32)
    lanes = slice(rank * N // world, (rank + 1) * N // world)
    adv = (ret[:-1, lanes] - val[:-1, lanes]).astype(np.float32)
    a64 = adv.astype(np.float64)
    stats = torch.tensor([adv.size, a64.mean(), ((a64 - a64.mean()) ** 2).sum()], dtype=torch.float64)
    _dist.allreduce_stats(stats)
    mean, std = _dist.stats_mean_std(*stats.tolist())
    norm = (adv - np.float32(mean)) / (np.float32(std) + np.float32(1e-5))
    full = O.normalize_advantages(ret, val)[:, lanes]
    # per-rank gradients -> all-reduce -> averaged clip + Adam
    P = 50
    g_local = torch.from_numpy(rng.standard_normal((world, P)).astype(np.float32)[rank] * 4)
    params = torch.from_numpy(np.linspace(-1, 1, P).astype(np.float32))
    _dist.broadcast_params(params)
    g = g_local.clone()
    scale = _dist.allreduce_grads(g)
    gmean = (g.numpy() * scale).astype(np.float64)
    # the bucketed form (tail reduced first, as the CNN engines do after the fc weight
    # gradient, then the head) gives the same sum
    gb = g_local.clone()
    assert _dist.start_bucket(gb[30:])
    assert _dist.allreduce_grads(gb) == scale   # reduces the head only
    assert torch.equal(gb, g)
    # a started bucket no allreduce_grads consumed (a minibatch that raised in between)
    # is forgotten by the next minibatch: the next gradient is reduced whole
    assert _dist.start_bucket(g_local.clone()[30:]) and _dist.pending_buckets() == 1
    _dist.begin_minibatch()
    assert _dist.pending_buckets() == 0
    gc = g_local.clone()
    _dist.allreduce_grads(gc)
    assert torch.equal(gc, g)
    # the optimizer-step guard is global: only rank 1 flags, both ranks see it
    flag = torch.zeros(1, dtype=torch.float64)
    _dist.global_guard(torch.tensor([0], dtype=torch.int32),
                       torch.tensor([1.0 if rank == 1 else 0.0], dtype=torch.float64), flag)
    assert flag.item() == 1.0
    _dist.global_guard(torch.tensor([7 if rank == 0 else 0], dtype=torch.int32),
                       torch.tensor([0.0], dtype=torch.float64), flag)
    assert flag.item() == 1.0
    _dist.global_guard(torch.tensor([0], dtype=torch.int32), torch.tensor([0.0], dtype=torch.float64), flag)
    assert flag.item() == 0.0
    p1, *_ = O.clip_adam(params.numpy().astype(np.float64), gmean, np.zeros(P), np.zeros(P), 1, 1e-3, 1e-5, 0.5)
    losses = torch.tensor([1.0 + rank, 2.0, 3.0], dtype=torch.float64)
    _dist.allreduce_losses(losses)
    out[rank] = (np.abs(norm - full).max(), p1, losses.numpy())
    dist.destroy_process_group()


def test_two_rank_protocol():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    err0, p0, l0 = out[0]
    err1, p1, l1 = out[1]
    assert err0 < 2e-6 and err1 < 2e-6          # global advantage normalisation
    assert np.array_equal(p0, p1)               # identical step on every rank
    assert np.allclose(l0, [1.5, 2.0, 3.0]) and np.allclose(l1, l0)


def test_welford_merge_large_mean_shards():
    """_dist.merge_moments (the rank merge of allreduce_stats, and the same update
    as the GPU kernels' mom_merge) on shards whose mean is 1e6 times their spread:
    count, mean and M2 match a two-pass float64 computation, where summed moments
    (Σx, Σx²) would lose the variance to cancellation."""
    from a2c_ppo_acktr import _dist
    rng = np.random.default_rng(3)
    shards = [1e5 + 0.01 * rng.standard_normal(n) for n in (1000, 37, 4096)]
    parts = [torch.tensor([s.size, s.mean(), ((s - s.mean()) ** 2).sum()], dtype=torch.float64) for s in shards]
    n, mean, m2 = _dist.merge_moments(parts).tolist()
    allx = np.concatenate(shards)
    ref_m2 = ((allx - allx.mean()) ** 2).sum()
    assert n == allx.size
    np.testing.assert_allclose(mean, allx.mean(), rtol=1e-15)
    np.testing.assert_allclose(m2, ref_m2, rtol=1e-9)
    naive = (allx ** 2).sum() - allx.sum() ** 2 / allx.size
    assert abs(naive - ref_m2) / ref_m2 > 1e-6   # what the summed-moment form would have lost
