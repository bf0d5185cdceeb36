"""RolloutStorage — drop-in for a2c_ppo_acktr/storage.py (reference
ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/storage.py:9-223).

Same constructor, public attributes (obs, vector_obs, recurrent_hidden_states,
rewards, value_preds, returns, action_log_probs, actions, masks, bad_masks,
num_steps, step) and methods.  Every per-step field is its own [T(+1), N, ...]
plane in HBM (structure of arrays); compute_returns, the minibatch gathers,
insert and after_update run as HIP kernels (libppo_hip.so) once the storage
has been moved to the MI355X with .to(device).  There is no CPU compute path.

Extensions (keyword-only, defaults keep the reference's behaviour):
  obs_dtype=torch.uint8  store observations as raw bytes (4x less HBM than the
                         reference's fp32); Policy decodes u8/255 inside conv1.
  device=...             allocate directly on the device (skips the host copy).
  gae_mode="exact"       compute_returns kernel: "exact" (default) walks each lane
                         sequentially in the reference's op order (bit-identical);
                         "scan" is the time-parallel affine scan (within fp32
                         tolerance; fills the GPU when there are few lanes, e.g.
                         c1's 8 or c2's 1024); "auto" picks scan below 16,384 lanes.
"""
import torch

from . import _dist
from ._hip import call, ptr, stream


def _flatten_helper(T, N, _tensor):
    # storage.py:5-6
    return _tensor.view(T * N, *_tensor.size()[2:])


class RolloutStorage(object):
    def __init__(self, num_steps, num_processes, obs_shape, vector_obs_shape, action_space,
                 recurrent_hidden_state_size, *, obs_dtype=torch.float32, device=None, gae_mode="exact"):
        if gae_mode not in ("exact", "scan", "auto"):
            raise ValueError(f"gae_mode {gae_mode!r}: 'exact', 'scan' or 'auto'")
        self.gae_mode = gae_mode
        kw = {} if device is None else {"device": device}
        self.obs = torch.zeros(num_steps + 1, num_processes, *obs_shape, dtype=obs_dtype, **kw)
        self.vector_obs = torch.zeros(num_steps + 1, num_processes, *vector_obs_shape, **kw)
        self.recurrent_hidden_states = torch.zeros(num_steps + 1, num_processes, recurrent_hidden_state_size, **kw)
        self.rewards = torch.zeros(num_steps, num_processes, 1, **kw)
        self.value_preds = torch.zeros(num_steps + 1, num_processes, 1, **kw)
        self.returns = torch.zeros(num_steps + 1, num_processes, 1, **kw)
        self.action_log_probs = torch.zeros(num_steps, num_processes, 1, **kw)
        if action_space.__class__.__name__ == 'Discrete':
            action_shape = 1
        else:
            action_shape = action_space.shape[0]
        self.actions = torch.zeros(num_steps, num_processes, action_shape, **kw)
        if action_space.__class__.__name__ == 'Discrete':
            self.actions = self.actions.long()
        self.masks = torch.ones(num_steps + 1, num_processes, 1, **kw)
        # Masks that indicate whether it's a true terminal state or time limit end state
        self.bad_masks = torch.ones(num_steps + 1, num_processes, 1, **kw)
        self.num_steps = num_steps
        self.step = 0
        self._adv = None          # raw then normalised advantages [T, N] (device)
        self._adv_partials = None
        self._adv_key = None      # (returns._version, value_preds._version) when _adv was produced
        self._adv_ready = False   # _adv holds the raw difference + matching partials

    # ------------------------------------------------------------------ moves
    def to(self, device):
        for name in ("obs", "vector_obs", "recurrent_hidden_states", "rewards", "value_preds", "returns",
                     "action_log_probs", "actions", "masks", "bad_masks"):
            setattr(self, name, getattr(self, name).to(device, non_blocking=True))
        self._adv = None
        self._adv_ready = False

    def half(self):
        """storage.py:48-58 (--half-precision, T/run.py:137-138): a float image
        observation plane becomes fp16, half the HBM of the reference's fp32 plane
        (u8 planes are already a quarter and stay bytes).  The per-step scalar
        planes (2 MB each at c3), vector obs and hidden states stay fp32 — GAE and
        the loss keep the reference's fp32 arithmetic — and actions stay int64;
        insert() converts fp16 masks / values written by the caller."""
        if self.obs.dtype.is_floating_point and self.obs.dim() >= 5:
            self.obs = self.obs.half()
        return self

    def _on_device(self):
        if not self.value_preds.is_cuda:
            raise RuntimeError("RolloutStorage lives on the host: move it to the MI355X with .to(device) "
                               "(the HIP engine has no CPU path)")

    # ----------------------------------------------------------------- insert
    def insert(self, obs, vector_obs, recurrent_hidden_states, actions, action_log_probs, value_preds, rewards,
               masks, bad_masks):
        """storage.py:60-73.  Bulk rows (obs, vector_obs, hxs) are copied unless the
        caller already wrote them in place; the six per-env scalars go in one kernel."""
        self._on_device()
        s, T, N = self.step, self.num_steps, self.rewards.shape[1]
        self._copy_row(self.obs[s + 1], obs, "obs")
        self._copy_row(self.vector_obs[s + 1], vector_obs, "vector_obs")
        self._copy_row(self.recurrent_hidden_states[s + 1], recurrent_hidden_states, "recurrent_hidden_states")
        dev = self.value_preds.device

        def col(x, dtype):
            if x is None:
                return None
            x = x.to(dev, dtype=dtype, non_blocking=True).reshape(-1)
            return x.contiguous()

        a = col(actions, self.actions.dtype)
        if self.actions.dtype != torch.int64 or self.actions.shape[2] != 1:
            self.actions[s].copy_(actions)   # Box/MultiBinary actions: plain copy
            a = None
        lp, v, r, m, bm = (col(action_log_probs, torch.float32), col(value_preds, torch.float32),
                           col(rewards, torch.float32), col(masks, torch.float32), col(bad_masks, torch.float32))
        call("ppo_storage_insert_scalars", N, s, ptr(a), ptr(lp), ptr(v), ptr(r), ptr(m), ptr(bm),
             self.actions.data_ptr(), self.action_log_probs.data_ptr(), self.value_preds.data_ptr(),
             self.rewards.data_ptr(), self.masks.data_ptr(), self.bad_masks.data_ptr(), stream())
        self.step = (self.step + 1) % self.num_steps
        self._adv_ready = False

    @staticmethod
    def _copy_row(dst, src, name):
        if src is None or dst.numel() == 0:
            return
        if src.data_ptr() == dst.data_ptr() and src.dtype == dst.dtype:
            return  # written in place (e.g. by the synthetic env kernel)
        if src.dtype != dst.dtype:
            if dst.dtype == torch.uint8:
                raise TypeError(f"{name}: u8 storage needs u8 frames (got {src.dtype}); construct the storage "
                                "with the default obs_dtype=torch.float32 for pre-normalised observations")
            src = src.to(dst.dtype)
        if not src.is_cuda:
            dst.copy_(src.reshape(dst.shape), non_blocking=True)   # host -> device transfer
            return
        src = src.contiguous()
        if src.numel() != dst.numel():
            raise RuntimeError(f"{name}: expected {tuple(dst.shape)}, got {tuple(src.shape)}")
        call("ppo_copy", dst.data_ptr(), src.data_ptr(), dst.numel() * dst.element_size(), stream())

    def after_update(self):
        """storage.py:75-80: slot T -> slot 0."""
        self._on_device()
        for t in (self.obs, self.vector_obs, self.recurrent_hidden_states, self.masks, self.bad_masks):
            if t.numel():
                call("ppo_copy", t[0].data_ptr(), t[-1].data_ptr(), t[0].numel() * t.element_size(), stream())

    # --------------------------------------------------------------- returns
    def compute_returns(self, next_value, use_gae, gamma, gae_lambda, use_proper_time_limits=True):
        """storage.py:82-121, one fused HIP kernel (bit-identical to the reference).
        Also produces the raw advantages and their moment partials for PPO.update."""
        self._on_device()
        T, N = self.rewards.shape[0], self.rewards.shape[1]
        nv = next_value.to(self.value_preds.device, torch.float32).reshape(-1).contiguous()
        if nv.numel() != N:
            raise RuntimeError(f"next_value has {nv.numel()} elements, expected {N}")
        self._ensure_adv(T, N)
        scan = self.gae_mode == "scan" or (self.gae_mode == "auto" and N < 16384)
        call("ppo_compute_returns_scan" if scan else "ppo_compute_returns", self.rewards.data_ptr(),
             self.value_preds.data_ptr(), self.masks.data_ptr(), self.bad_masks.data_ptr(), nv.data_ptr(),
             self.returns.data_ptr(), self._adv.data_ptr(), self._adv_partials.data_ptr(), T, N, float(gamma),
             float(gae_lambda), int(bool(use_gae)), int(bool(use_proper_time_limits)), stream())
        self._adv_key = (self.returns._version, self.value_preds._version)
        self._adv_ready = True
        self._adv_nparts = call("ppo_gae_scan_partials_count" if scan else "ppo_gae_partials_count", N)

    def _ensure_adv(self, T, N):
        dev = self.value_preds.device
        nparts = max(call("ppo_gae_partials_count", N), call("ppo_gae_scan_partials_count", N),
                     call("ppo_adv_diff_partials_count", T * N))
        if self._adv is None or self._adv.shape != (T, N) or self._adv.device != dev:
            self._adv = torch.empty(T, N, device=dev)
            self._adv_partials = torch.empty(3 * nparts, dtype=torch.float64, device=dev)
            self._adv_stats = torch.empty(3, dtype=torch.float64, device=dev)

    def normalized_advantages(self):
        """algo/ppo.py:35-37: (adv - mean) / (std + 1e-5) over all T*N samples —
        across every rank when torch.distributed is initialised (one 3-double
        all-reduce), so sharded lanes see single-GPU statistics.  Returns [T, N]."""
        self._on_device()
        T, N = self.rewards.shape[0], self.rewards.shape[1]
        self._ensure_adv(T, N)
        key = (self.returns._version, self.value_preds._version)
        if not (self._adv_ready and self._adv_key == key):
            n = T * N
            call("ppo_adv_diff", self.returns.data_ptr(), self.value_preds.data_ptr(), self._adv.data_ptr(),
                 self._adv_partials.data_ptr(), n, stream())
            self._adv_nparts = call("ppo_adv_diff_partials_count", n)
        call("ppo_adv_finalize", self._adv_partials.data_ptr(), self._adv_nparts, float(T * N),
             self._adv_stats.data_ptr(), stream())
        _dist.allreduce_stats(self._adv_stats)
        call("ppo_adv_normalize", self._adv.data_ptr(), T * N, self._adv_stats.data_ptr(), stream())
        self._adv_ready = False   # _adv now holds normalised values
        return self._adv

    # ------------------------------------------------------------ generators
    def _gather(self, plane, idx, rows_shape):
        out = torch.empty(idx.numel(), *rows_shape, dtype=plane.dtype, device=plane.device)
        row_bytes = plane[0].numel() // plane.shape[1] * plane.element_size() if plane.dim() > 1 else 0
        if out.numel():
            call("ppo_gather_rows", plane.data_ptr(), idx.data_ptr(), out.data_ptr(), idx.numel(),
                 row_bytes, stream())
        return out

    def feed_forward_generator(self, advantages, num_mini_batch=None, mini_batch_size=None):
        """storage.py:123-160.  The permutation is torch.randperm on the default CPU
        generator — the very call SubsetRandomSampler makes in the reference — so the
        minibatch index sets are bit-identical; the row gathers run on the GPU."""
        num_steps, num_processes = self.rewards.size()[0:2]
        batch_size = num_processes * num_steps
        if mini_batch_size is None:
            assert batch_size >= num_mini_batch, (
                "PPO requires the number of processes ({}) "
                "* number of steps ({}) = {} "
                "to be greater than or equal to the number of PPO mini batches ({})."
                "".format(num_processes, num_steps, num_processes * num_steps, num_mini_batch))
            mini_batch_size = batch_size // num_mini_batch
        self._on_device()
        perm = torch.randperm(batch_size).to(self.value_preds.device, non_blocking=True)
        dev = self.value_preds.device
        for start in range(0, batch_size - mini_batch_size + 1, mini_batch_size):
            idx = perm[start:start + mini_batch_size]
            obs_batch = self._gather(self.obs, idx, self.obs.shape[2:])
            vector_obs_batch = self._gather(self.vector_obs, idx, self.vector_obs.shape[2:])
            hxs_batch = self._gather(self.recurrent_hidden_states, idx, self.recurrent_hidden_states.shape[2:])
            actions_batch = self._gather(self.actions, idx, (self.actions.size(-1),))
            value_preds_batch = self._gather(self.value_preds, idx, (1,))
            return_batch = self._gather(self.returns, idx, (1,))
            masks_batch = self._gather(self.masks, idx, (1,))
            old_action_log_probs_batch = self._gather(self.action_log_probs, idx, (1,))
            if advantages is None:
                adv_targ = None
            else:
                adv = advantages.to(dev).reshape(num_steps, num_processes, 1).contiguous()
                adv_targ = self._gather(adv, idx, (1,))
            yield obs_batch, vector_obs_batch, hxs_batch, actions_batch, \
                value_preds_batch, return_batch, masks_batch, old_action_log_probs_batch, adv_targ

    def _gather_cols(self, plane, envs, T, rows_shape):
        n = envs.numel()
        out = torch.empty(T, n, *rows_shape, dtype=plane.dtype, device=plane.device)
        row_bytes = plane[0, 0].numel() * plane.element_size()
        if out.numel():
            call("ppo_gather_env_columns", plane.data_ptr(), envs.data_ptr(), out.data_ptr(), T, plane.shape[1], n,
                 row_bytes, stream())
        return out

    def recurrent_generator(self, advantages, num_mini_batch):
        """storage.py:162-223: whole env sequences, env order from torch.randperm(N)."""
        self._on_device()
        num_processes = self.rewards.size(1)
        assert num_processes >= num_mini_batch, (
            "PPO requires the number of processes ({}) "
            "to be greater than or equal to the number of "
            "PPO mini batches ({}).".format(num_processes, num_mini_batch))
        num_envs_per_batch = num_processes // num_mini_batch
        perm = torch.randperm(num_processes)
        dev = self.value_preds.device
        T = self.num_steps
        for start_ind in range(0, num_processes, num_envs_per_batch):
            if start_ind + num_envs_per_batch > num_processes:
                # the reference indexes perm past its end here (storage.py:181-182)
                raise IndexError("index {} is out of bounds for dimension 0 with size {}".format(
                    num_processes, num_processes))
            envs = perm[start_ind:start_ind + num_envs_per_batch].to(dev)
            N = num_envs_per_batch
            obs_batch = self._gather_cols(self.obs, envs, T, self.obs.shape[2:])
            vector_obs_batch = self._gather_cols(self.vector_obs, envs, T, self.vector_obs.shape[2:])
            hxs_batch = self._gather_cols(self.recurrent_hidden_states, envs, 1,
                                          self.recurrent_hidden_states.shape[2:]).view(N, -1)
            actions_batch = self._gather_cols(self.actions, envs, T, (self.actions.size(-1),))
            value_preds_batch = self._gather_cols(self.value_preds, envs, T, (1,))
            return_batch = self._gather_cols(self.returns, envs, T, (1,))
            masks_batch = self._gather_cols(self.masks, envs, T, (1,))
            old_action_log_probs_batch = self._gather_cols(self.action_log_probs, envs, T, (1,))
            adv = advantages.to(dev).reshape(T, num_processes, 1).contiguous()
            adv_targ = self._gather_cols(adv, envs, T, (1,))
            yield (_flatten_helper(T, N, obs_batch), _flatten_helper(T, N, vector_obs_batch), hxs_batch,
                   _flatten_helper(T, N, actions_batch), _flatten_helper(T, N, value_preds_batch),
                   _flatten_helper(T, N, return_batch), _flatten_helper(T, N, masks_batch),
                   _flatten_helper(T, N, old_action_log_probs_batch), _flatten_helper(T, N, adv_targ))
