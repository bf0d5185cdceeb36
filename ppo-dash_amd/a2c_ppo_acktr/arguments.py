"""Legacy argument parser (reference a2c_ppo_acktr/arguments.py:6-161).  run.py
imports get_args but parses with make_env.otc_arg_parser; the PPO-relevant
flags and defaults are kept here for scripts that still call it."""
import argparse

import torch


def get_args(argv=None):
    p = argparse.ArgumentParser(description='RL')
    p.add_argument('--algo', default='a2c', help='algorithm to use: a2c | ppo | acktr')
    p.add_argument('--lr', type=float, default=7e-4)
    p.add_argument('--eps', type=float, default=1e-5)
    p.add_argument('--alpha', type=float, default=0.99)
    p.add_argument('--gamma', type=float, default=0.99)
    p.add_argument('--use-gae', action='store_true', default=False)
    p.add_argument('--gae-lambda', type=float, default=0.95)
    p.add_argument('--entropy-coef', type=float, default=0.01)
    p.add_argument('--value-loss-coef', type=float, default=0.5)
    p.add_argument('--max-grad-norm', type=float, default=0.5)
    p.add_argument('--seed', type=int, default=1)
    p.add_argument('--cuda-deterministic', action='store_true', default=False)
    p.add_argument('--num-processes', type=int, default=16)
    p.add_argument('--num-steps', type=int, default=5)
    p.add_argument('--ppo-epoch', type=int, default=4)
    p.add_argument('--num-mini-batch', type=int, default=32)
    p.add_argument('--clip-param', type=float, default=0.2)
    p.add_argument('--log-interval', type=int, default=10)
    p.add_argument('--save-interval', type=int, default=100)
    p.add_argument('--eval-interval', type=int, default=None)
    p.add_argument('--num-env-steps', type=int, default=10e6)
    p.add_argument('--env-name', default='PongNoFrameskip-v4')
    p.add_argument('--log-dir', default='/tmp/gym/')
    p.add_argument('--save-dir', default='./trained_models/')
    p.add_argument('--no-cuda', action='store_true', default=False)
    p.add_argument('--use-proper-time-limits', action='store_true', default=False)
    p.add_argument('--recurrent-policy', action='store_true', default=False)
    p.add_argument('--use-linear-lr-decay', action='store_true', default=False)
    args = p.parse_args(argv)
    args.cuda = not args.no_cuda and torch.cuda.is_available()
    assert args.algo in ['a2c', 'ppo', 'acktr']
    if args.recurrent_policy:
        assert args.algo in ['a2c', 'ppo'], 'Recurrent policy is not implemented for ACKTR'
    return args
