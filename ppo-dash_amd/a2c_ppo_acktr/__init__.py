"""MI355X-native drop-in for the `a2c_ppo_acktr` package used by ppo-dash
(reference: ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/).

Put `ppo-dash_amd/` on sys.path in place of the reference tree; `run.py`'s
imports (`from a2c_ppo_acktr import algo, utils`, `...model import Policy,
CNNBase`, `...storage import RolloutStorage`, ...) resolve here.  The hot path
(RolloutStorage, Policy, PPO.update) runs as HIP kernels in libppo_hip.so.
"""
