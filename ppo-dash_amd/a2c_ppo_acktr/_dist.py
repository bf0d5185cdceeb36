"""The multi-GPU protocol (new design: the reference's PPO path has no
collectives).  One process per GPU, each owning N/G env
lanes and its own RolloutStorage; torch.distributed with backend "nccl" is
RCCL over xGMI on ROCm.  Exchanges, all on the current stream:

  once per run     broadcast_params   rank 0's flat parameters to every rank
  once per update  allreduce_stats    {count, mean, M2} (3 doubles) gathered from
                                      every rank and merged in rank order (Chan
                                      et al.) -> global advantage mean / unbiased
                                      std (ppo.py:36; Welford)
  per minibatch    allreduce_grads    Σ of the flat fp32 gradient; clip + Adam
                                      then run on Σ/G (scale returned here) —
                                      CNN policies in two buckets: the fc + heads
                                      tail (92 % of the bytes, final once the fc
                                      weight gradient is reduced) on a side stream,
                                      overlapped with the conv backward, then the
                                      conv head of the buffer (start_bucket, then
                                      allreduce_grads finishes the buffer)
  once per update  allreduce_losses   mean of the 3 logged losses over ranks

These helpers are plain torch.distributed calls so they run unchanged under
gloo on CPU tensors (tests/test_dist_gloo.py) and under RCCL on the MI355X.

force_collectives(True) runs every exchange even at world size 1 (a one-rank
RCCL communicator: bench.py --force-collectives), so the RCCL path — stream
ordering against the engine's raw-stream launches included — executes on a
one-GPU box; a one-rank sum is exact, so results are bit-identical to the
collective-free path.  time_grads(True) records HIP events around every
gradient all-reduce on the current stream (the one the engine launches on).
"""
import math

import torch
import torch.distributed as dist

_FORCE = False
_TIMING = {"on": False, "events": []}


def force_collectives(on=True):
    global _FORCE
    _FORCE = bool(on)


def world_size():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def active():
    """collectives run: torch.distributed initialised and more than one rank, or forced"""
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _FORCE)


def broadcast_params(flat):
    if active():
        dist.broadcast(flat, src=0)


def merge_moments(parts):
    """Chan et al.'s pairwise merge of (count, mean, M2) triples in the given
    order — the same update the GPU kernels use (gae.hip mom_merge), on tensors
    of the caller's device (no host synchronisation)."""
    n, mean, m2 = parts[0][0], parts[0][1], parts[0][2]
    for p in parts[1:]:
        nb, mb, qb = p[0], p[1], p[2]
        tot = n + nb
        f = torch.where(tot > 0, nb / torch.where(tot > 0, tot, torch.ones_like(tot)), torch.zeros_like(tot))
        d = mb - mean
        mean = mean + d * f
        m2 = m2 + qb + d * d * n * f
        n = tot
    return torch.stack([n, mean, m2])


def allreduce_stats(stats):
    """stats {count, mean, M2} of this rank's advantages -> the global ones, on
    every rank bit-identically (all ranks merge the same gathered list in rank
    order); a Welford merge instead of summed moments, so a shard whose mean is
    large against its spread loses no precision"""
    if active():
        parts = [torch.empty_like(stats) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, stats)
        stats.copy_(merge_moments(parts))
    return stats


def time_grads(on=True):
    """start (clearing) / stop event timing of allreduce_grads"""
    _TIMING["on"] = bool(on)
    if on:
        _TIMING["events"] = []


def grad_allreduce_times():
    """[(ms, bytes)] of the timed gradient all-reduces (synchronises the events)"""
    out = []
    for e0, e1, nbytes in _TIMING["events"]:
        e1.synchronize()
        out.append((e0.elapsed_time(e1), nbytes))
    return out


def _timed_all_reduce(t):
    if _TIMING["on"]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dist.all_reduce(t)
        e1.record()
        _TIMING["events"].append((e0, e1, t.numel() * t.element_size()))
    else:
        dist.all_reduce(t)


_OVERLAP = {"on": True, "stream": {}}
# started tail buckets of the CURRENT minibatch: end address of the tail -> (event or
# None, element count); allreduce_grads of a buffer ending there waits for it and
# reduces only the rest, so no caller can sum a tail twice.  begin_minibatch() drops
# entries a failed minibatch left behind (after the current stream has waited for
# their collectives), so a later buffer at the same address never matches a stale one.
_PENDING = {}


def begin_minibatch():
    """Called by the engines before a minibatch's backward: joins and forgets any
    tail bucket that no allreduce_grads consumed (an exception between
    start_bucket and the optimizer step).  Its side-stream collective still writes
    into the gradient buffer, so the current stream waits for it first."""
    for done, _ in _PENDING.values():
        if done is not None:
            torch.cuda.current_stream().wait_event(done)
    _PENDING.clear()


def pending_buckets():
    """number of started tail buckets not yet joined into the current stream"""
    return len(_PENDING)


def assert_no_pending(what):
    """Persistent GRU launches need all their blocks co-resident: a collective
    kernel running beside them on a side stream could hold CUs they wait for.
    Every started bucket is joined (current stream waits for its event) in
    allreduce_grads before clip + Adam, so none may be pending when such a
    launch is queued on the current stream."""
    if _PENDING:
        raise RuntimeError(f"{what}: {len(_PENDING)} gradient bucket(s) still reducing on a side stream")


def overlap_buckets(on=True):
    """enable / disable the bucketed gradient all-reduce (start_bucket)"""
    _OVERLAP["on"] = bool(on)


def _end(t):
    return t.data_ptr() + t.numel() * t.element_size()


def start_bucket(tail):
    """Start the all-reduce of a finished tail of the flat gradient on a side
    stream, ordered after everything queued so far on the current stream (the
    kernels that wrote it); the current stream goes on with the rest of the
    backward, and the next allreduce_grads of the buffer that ends with this tail
    waits for it and reduces only the head.  No-op without collectives."""
    if not active() or not _OVERLAP["on"]:
        return False
    if not tail.is_cuda:   # host tensors (gloo): reduced in place now, only the split remains
        _timed_all_reduce(tail)
        _PENDING[_end(tail)] = (None, tail.numel())
        return True
    cur = torch.cuda.current_stream(tail.device)
    side = _OVERLAP["stream"].get(tail.device)
    if side is None:
        side = _OVERLAP["stream"][tail.device] = torch.cuda.Stream(tail.device)
    ready = torch.cuda.Event()
    ready.record(cur)
    side.wait_event(ready)
    with torch.cuda.stream(side):
        _timed_all_reduce(tail)
        done = torch.cuda.Event()
        done.record(side)
    _PENDING[_end(tail)] = (done, tail.numel())
    return True


def allreduce_grads(grad):
    """Sum the flat gradient over ranks; returns the scale (1/G) that turns it
    into the mean, applied inside the clip + Adam kernels.  A tail of grad already
    started by start_bucket is waited for (on the current stream), not reduced again."""
    G = world_size()
    if active():
        pending = _PENDING.pop(_end(grad), None)
        if pending is not None and pending[1] <= grad.numel():
            done, n = pending
            if done is not None:
                torch.cuda.current_stream(grad.device).wait_event(done)
            if grad.numel() > n:
                _timed_all_reduce(grad[:grad.numel() - n])
        else:
            _timed_all_reduce(grad)
    return 1.0 / G


def global_guard(err, bad, out):
    """The optimizer-step guard made global (G > 1): out (float64 [1], device) =
    Σ over ranks of (err != 0) + bad, where err is this rank's persistent-GRU error
    word (int32 view) and bad its count of out-of-range stored actions (float64
    view).  The gradient the step consumes is already summed over ranks, so a
    failure on ANY rank must skip the step on EVERY rank; clip + Adam read out
    (> 0 skips).  Both terms are >= 0, so the sum is > 0 iff some rank failed."""
    torch.add(bad, (err != 0).to(torch.float64), out=out)
    if active():
        dist.all_reduce(out)
    return out


def allreduce_losses(acc):
    G = world_size()
    if active():
        dist.all_reduce(acc)
        acc /= G
    return acc


def stats_mean_std(count, mean, m2):
    """Host restatement of adv_normalize_kernel's statistics (gae.hip)."""
    var = max(m2 / (count - 1.0), 0.0)
    return mean, math.sqrt(var)
