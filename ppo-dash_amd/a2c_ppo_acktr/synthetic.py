"""Synthetic vectorised environment on the GPU.

Stands in for the reference's VecPyTorch + ShmemVecEnv + Unity simulator
(T/make_env.py:58-114, T/sohojoe_shmem_vec_env.py:23-142), which are outside
this engine's scope: one kernel writes the next u8 observation of every lane
straight into its RolloutStorage slot, plus rewards U[0,1), done ~
Bernoulli(p_done) -> masks, and bad_masks = 1.  Observations are a counter-based
hash of (seed, step, lane, byte), so any run is reproducible on the host
(tests/test_gpu_storage.py restates it in numpy).
"""
import torch

from ._hip import call, stream


class Discrete(object):
    """duck-typed gym.spaces.Discrete (storage.py:20, model.py:30)"""

    def __init__(self, n):
        self.n = n
        self.shape = ()


class SyntheticVecEnv(object):
    def __init__(self, num_envs, obs_shape=(4, 84, 84), num_actions=8, seed=123, p_done=0.01, device=None):
        self.num_envs = num_envs
        self.obs_shape = tuple(obs_shape)
        self.action_space = Discrete(num_actions)
        self.vector_obs_len = 0
        self.seed = int(seed)
        self.p_done = float(p_done)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.counter = 0
        self.obs_bytes = 1
        for d in self.obs_shape:
            self.obs_bytes *= d
        self.reward = torch.zeros(num_envs, 1, device=self.device)
        self.mask = torch.ones(num_envs, 1, device=self.device)
        self.bad_mask = torch.ones(num_envs, 1, device=self.device)

    def _write(self, obs_slot, reward, mask, bad_mask):
        if obs_slot.dtype != torch.uint8 or not obs_slot.is_contiguous():
            raise TypeError("SyntheticVecEnv writes u8 frames into a contiguous uint8 slot")
        call("ppo_synth_env_step", obs_slot.data_ptr(), self.num_envs, self.obs_bytes,
             None if reward is None else reward.data_ptr(), None if mask is None else mask.data_ptr(),
             None if bad_mask is None else bad_mask.data_ptr(), self.seed, self.counter, self.p_done, stream())
        self.counter += 1

    def reset_into(self, obs_slot):
        self._write(obs_slot, None, None, None)

    def step_into(self, obs_slot, action=None):
        """Writes the next observation into obs_slot ([N,C,H,W] u8) and returns
        (reward [N,1], masks [N,1], bad_masks [N,1]) device tensors.  The synthetic
        dynamics ignore the action (fixed-shape synthetic workload)."""
        self._write(obs_slot, self.reward, self.mask, self.bad_mask)
        return self.reward, self.mask, self.bad_mask


class CartPoleVecEnv(object):
    """CartPole-v1 on the GPU for the MLPBase workload (SURVEY.md §8 c1 —
    the reference trains it through gym + VecPyTorch, T/envs.py:40-96).

    gym's dynamics (Euler, tau 0.02, force ±10, |x| > 2.4 or |theta| > 12°
    terminates, reward 1 every step) in fp32, TimeLimit(max_steps) marks a
    bad transition (bad_mask 0), and every ended lane resets to U(-0.05, 0.05)^4
    drawn from the counter RNG, as baselines' auto-resetting VecEnv does.
    `ep_len[n]` is the finished episode's length on the step it ended, else 0
    (what the reference's `info['episode']['r']` carries for CartPole)."""

    def __init__(self, num_envs, seed=123, max_steps=500, device=None):
        self.num_envs = num_envs
        self.obs_shape = (4,)
        self.action_space = Discrete(2)
        self.vector_obs_len = 0
        self.seed = int(seed)
        self.max_steps = int(max_steps)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.counter = 0
        self.state = torch.zeros(num_envs, 4, device=self.device)
        self.steps = torch.zeros(num_envs, dtype=torch.int32, device=self.device)
        self.reward = torch.zeros(num_envs, 1, device=self.device)
        self.mask = torch.ones(num_envs, 1, device=self.device)
        self.bad_mask = torch.ones(num_envs, 1, device=self.device)
        self.ep_len = torch.zeros(num_envs, device=self.device)

    def _check(self, obs_slot):
        if obs_slot.dtype != torch.float32 or not obs_slot.is_contiguous() or obs_slot.numel() != 4 * self.num_envs:
            raise TypeError("CartPoleVecEnv writes float32 [N,4] observations into a contiguous slot")

    def reset_into(self, obs_slot):
        self._check(obs_slot)
        call("ppo_cartpole_step", self.state.data_ptr(), self.steps.data_ptr(), None, obs_slot.data_ptr(), None, None,
             None, None, self.num_envs, self.seed, self.counter, self.max_steps, stream())
        self.counter += 1

    def step_into(self, obs_slot, action):
        """Applies action ([N,1] int64, device) and writes the next observation into
        obs_slot; returns (reward [N,1], masks [N,1], bad_masks [N,1])."""
        self._check(obs_slot)
        action = action.reshape(-1)
        if action.dtype != torch.int64 or action.numel() != self.num_envs or not action.is_cuda:
            raise TypeError("CartPoleVecEnv.step_into expects [N,1] int64 device actions")
        call("ppo_cartpole_step", self.state.data_ptr(), self.steps.data_ptr(), action.contiguous().data_ptr(),
             obs_slot.data_ptr(), self.reward.data_ptr(), self.mask.data_ptr(), self.bad_mask.data_ptr(),
             self.ep_len.data_ptr(), self.num_envs, self.seed, self.counter, self.max_steps, stream())
        self.counter += 1
        return self.reward, self.mask, self.bad_mask
