"""The multi-GPU protocol (new design: the reference's PPO path has no
collectives).  One process per GPU, each owning N/G env
lanes and its own RolloutStorage; torch.distributed with backend "nccl" is
RCCL over xGMI on ROCm.  Exchanges, all on the current stream:

  once per run     broadcast_params   rank 0's flat parameters to every rank
  once per update  allreduce_stats    {count, Σadv, Σadv²} (3 doubles) -> global
                                      advantage mean / unbiased std (ppo.py:36)
  per minibatch    allreduce_grads    Σ of the flat fp32 gradient; clip + Adam
                                      then run on Σ/G (scale returned here)
  once per update  allreduce_losses   mean of the 3 logged losses over ranks

These helpers are plain torch.distributed calls so they run unchanged under
gloo on CPU tensors (tests/test_dist_gloo.py) and under RCCL on the MI355X.
"""
import math

import torch.distributed as dist


def world_size():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def broadcast_params(flat):
    if world_size() > 1:
        dist.broadcast(flat, src=0)


def allreduce_stats(stats):
    if world_size() > 1:
        dist.all_reduce(stats)
    return stats


def allreduce_grads(grad):
    """Sum the flat gradient over ranks; returns the scale (1/G) that turns it
    into the mean, applied inside the clip + Adam kernels."""
    G = world_size()
    if G > 1:
        dist.all_reduce(grad)
    return 1.0 / G


def allreduce_losses(acc):
    G = world_size()
    if G > 1:
        dist.all_reduce(acc)
        acc /= G
    return acc


def stats_mean_std(count, s, q):
    """Host restatement of adv_normalize_kernel's statistics (gae.hip)."""
    mean = s / count
    var = max((q - s * mean) / (count - 1.0), 0.0)
    return mean, math.sqrt(var)
