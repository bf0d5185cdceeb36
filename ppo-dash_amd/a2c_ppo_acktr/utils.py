"""Helpers — drop-in for a2c_ppo_acktr/utils.py (reference
ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/utils.py:1-65)."""
import glob
import os

import torch
import torch.nn as nn

from .envs import VecNormalize


def get_render_func(venv):
    """utils.py:11-19: walk .envs / .venv / .env wrappers to a render function."""
    for attr in ("envs", "venv", "env"):
        if hasattr(venv, attr):
            inner = getattr(venv, attr)
            return inner[0].render if attr == "envs" else get_render_func(inner)
    return None


def get_vec_normalize(venv):
    """utils.py:22-28."""
    while venv is not None:
        if isinstance(venv, VecNormalize):
            return venv
        venv = getattr(venv, "venv", None)
    return None


class AddBias(nn.Module):
    """utils.py:32-43 (kept for DiagGaussian's log-std)."""

    def __init__(self, bias):
        super(AddBias, self).__init__()
        self._bias = nn.Parameter(bias.unsqueeze(1))

    def forward(self, x):
        shape = (1, -1) if x.dim() == 2 else (1, -1, 1, 1)
        return x + self._bias.t().view(*shape)


def update_linear_schedule(optimizer, epoch, total_num_epochs, initial_lr):
    """utils.py:46-50: lr decays linearly to 0 over total_num_epochs updates."""
    lr = initial_lr - (initial_lr * (epoch / float(total_num_epochs)))
    for param_group in optimizer.param_groups:
        param_group['lr'] = lr


def init(module, weight_init, bias_init, gain=1):
    """utils.py:53-56."""
    weight_init(module.weight.data, gain=gain)
    bias_init(module.bias.data)
    return module


def cleanup_log_dir(log_dir):
    """utils.py:59-65."""
    os.makedirs(log_dir, exist_ok=True)
    for f in glob.glob(os.path.join(log_dir, '*.monitor.csv')):
        os.remove(f)
