"""Vec-env boundary on the MI355X.

Reference (ppo-dash-study/013_…/ unless noted; T/make_env.py:58-114 holds the
same VecPyTorch):
  * VecPyTorch                 pytorch_wrappers.py:105-160
  * VecPyTorchFrameStack       pytorch_wrappers.py:58-102
  * NormalizeWrapper           sohojoe_wrappers.py:855-884 (per-env, in the env workers)
  * FrameStackMono(k=2)        sohojoe_wrappers.py:425-501 (per-env)
  * TransposeImage             pytorch_wrappers.py:170-203 (per-env)

The reference converts every frame to float64 in each env worker (normalise,
grey plane, transpose), ships 4 x 84 x 84 x 8 bytes per env-step through shared
memory, casts to fp32 on the host and copies that over PCIe.  Here the env side
ships the raw u8 RGB frame (84 x 84 x 3 bytes, 10.7 x fewer), VecPyTorch moves it
through a pinned staging buffer with one asynchronous host->device copy, and
ObsPreprocess does normalise + grey + transpose + fp32 in one HIP kernel
(ppo_obs_preprocess), bit-identical to the reference chain (see tests).
VecPyTorchFrameStack keeps the stack on the device and updates it in place with
one kernel (ppo_frame_stack) instead of a slice copy plus a Python loop over envs.
"""
import numpy as np
import torch

from ._hip import call, require_device, stream


class ObsPreprocess(object):
    """NormalizeWrapper -> FrameStackMono(2) -> TransposeImage -> .float(), fused.

    mode: "raw" (values as they are), "div255" (NormalizeWrapper without a file:
    u8 / 255), "norm" ((u8 - mean) / std with mean [S][S][3], std a scalar, as
    NormalizeWrapper(env, "ObtRetro-v6") loads them).  mono: append the grey
    plane FrameStackMono(env, 2) adds (4 channels), else 3 channels."""

    def __init__(self, size=84, mode="div255", mean=None, std=None, mono=True, device=None):
        if mode not in ("raw", "div255", "norm"):
            raise ValueError(mode)
        if mode == "norm" and (mean is None or std is None):
            raise ValueError("mode 'norm' needs mean and std")
        require_device()
        self.size, self.mode, self.mono = int(size), mode, bool(mono)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.channels = 4 if mono else 3
        self.mean = None
        self.std = 0.0
        if mode == "norm":
            m = np.asarray(mean, dtype=np.float64).reshape(self.size, self.size, 3)
            self.mean = torch.from_numpy(np.ascontiguousarray(m)).to(self.device)
            s = np.asarray(std, dtype=np.float64)
            if s.size != 1:
                raise ValueError("std must be a scalar (ObtRetro-v6_std.txt holds one value)")
            self.std = float(s.reshape(()))

    @classmethod
    def from_files(cls, prefix, size=84, mono=True, device=None):
        """NormalizeWrapper(env, prefix): np.loadtxt(prefix + '_mean.txt' / '_std.txt')"""
        return cls(size, "norm", np.loadtxt(prefix + "_mean.txt"), np.loadtxt(prefix + "_std.txt"), mono, device)

    def __call__(self, frames, out=None):
        """frames: u8 [N][S][S][3] on the device -> fp32 [N][C][S][S] (or into out,
        any [N][C][S][S] fp32 view whose env rows are contiguous, e.g. rollouts.obs[k])"""
        S = self.size
        if frames.dtype != torch.uint8 or frames.device != self.device or tuple(frames.shape[1:]) != (S, S, 3):
            raise TypeError("ObsPreprocess wants u8 [N][%d][%d][3] frames on %s" % (S, S, self.device))
        frames = frames.contiguous()
        N = frames.shape[0]
        if out is None:
            out = torch.empty(N, self.channels, S, S, device=self.device)
        if out.dtype != torch.float32 or tuple(out.shape) != (N, self.channels, S, S) or (N and not out[0].is_contiguous()):
            raise TypeError("ObsPreprocess: out must be fp32 [%d][%d][%d][%d] with contiguous env rows"
                            % (N, self.channels, S, S))
        if N == 0:
            return out
        mode = {"raw": 0, "div255": 1, "norm": 2}[self.mode]
        call("ppo_obs_preprocess", frames.data_ptr(), S * S * 3, N, S, mode,
             None if self.mean is None else self.mean.data_ptr(), self.std, int(self.mono), out.data_ptr(),
             out.stride(0), stream())
        return out


class _Staging(object):
    """pinned host buffer reused across steps; the H2D copy runs on the current
    stream and the buffer is only rewritten after that copy has completed"""

    def __init__(self):
        self.buf = None
        self.event = None

    def upload(self, arr, device):
        src = torch.from_numpy(np.ascontiguousarray(arr))
        if self.buf is None or self.buf.dtype != src.dtype or self.buf.numel() < src.numel():
            self.buf = torch.empty(src.numel(), dtype=src.dtype).pin_memory()
            self.event = None
        if self.event is not None:
            self.event.synchronize()   # the previous step's copy out of this buffer is done
        host = self.buf[:src.numel()].view(src.shape)
        host.copy_(src)
        dev = torch.empty(src.shape, dtype=src.dtype, device=device)
        dev.copy_(host, non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record()
        return dev


class VecPyTorch(object):
    """pytorch_wrappers.py:105-160 with the same reset / step_async / step_wait.

    venv: a baselines-style vec env (reset() -> obs, step_async(actions),
    step_wait() -> (obs, reward, done, info)); obs either an array or a dict
    with 'visual' and 'vector'.  preprocess: an ObsPreprocess applied on the
    device to raw u8 [N][S][S][3] visual frames (the env-side normalise/grey/
    transpose wrappers moved onto the GPU); without it visual obs are copied as
    they come and cast to fp32 (fp16 with half_precision) on the device."""

    def __init__(self, venv, device, half_precision=False, preprocess=None, fused=False):
        """fused=True: hand the raw u8 RGB frames on unchanged ([N][S][S][3], 21 KB
        per frame in HBM) for a policy that decodes them inside conv1
        (Policy.set_obs_decode(preprocess)); store them in a
        RolloutStorage(..., (S, S, 3), ..., obs_dtype=torch.uint8)."""
        if fused and preprocess is None:
            raise ValueError("fused=True needs the preprocess the policy decodes with")
        self.fused = bool(fused)
        self.venv = venv
        self.num_envs = venv.num_envs
        self.device = device
        self._half_precision = half_precision
        self.preprocess = preprocess
        self.observation_space = venv.observation_space
        self.action_space = getattr(venv, "action_space", None)
        self._vector_obs_len = 0
        self._has_vector_obs = hasattr(self.observation_space, "spaces")
        if self._has_vector_obs:
            self._vector_obs_len = self.observation_space.spaces["vector"].shape[0]
            self.observation_space = self.observation_space.spaces["visual"]
        self._stage = {"visual": _Staging(), "vector": _Staging()}

    @property
    def vector_obs_len(self):
        return self._vector_obs_len

    def _convert(self, obs):
        vector_obs = np.zeros(0, np.float16 if self._half_precision else np.float32)
        if self._has_vector_obs:
            vector_obs = obs["vector"]
            obs = obs["visual"]
        dt = torch.float16 if self._half_precision else torch.float32
        vis = self._stage["visual"].upload(obs, self.device)   # u8 frames cross PCIe as u8
        if self.fused:
            pass   # raw frames: the policy's conv1 applies the decode
        elif self.preprocess is not None:
            vis = self.preprocess(vis)
            if self._half_precision:
                vis = vis.half()
        else:
            vis = vis.to(dt)
        vec = self._stage["vector"].upload(np.asarray(vector_obs), self.device).to(dt)
        return vis, vec

    def reset(self):
        return self._convert(self.venv.reset())

    def step_async(self, actions):
        if isinstance(actions, torch.LongTensor):   # as the reference: only CPU LongTensors are squeezed
            actions = actions.squeeze(1)
        self.venv.step_async(actions.cpu().numpy())

    def step_wait(self):
        obs, reward, done, info = self.venv.step_wait()
        vis, vec = self._convert(obs)
        reward = torch.from_numpy(np.asarray(reward)).unsqueeze(dim=1).float()
        return vis, vec, reward, done, info

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        if hasattr(self.venv, "close"):
            self.venv.close()


class VecPyTorchFrameStack(object):
    """pytorch_wrappers.py:58-102: stacked obs [N][nstack*C][...] on the device,
    updated in place by ppo_frame_stack (shift, zero finished envs, append)."""

    def __init__(self, venv, nstack, device=None):
        require_device()
        self.venv = venv
        self.nstack = nstack
        self.num_envs = venv.num_envs
        wos = venv.observation_space
        self.shape_dim0 = wos.shape[0]
        self.frame_shape = tuple(wos.shape)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.stacked_obs = torch.zeros((venv.num_envs, nstack * self.shape_dim0) + self.frame_shape[1:], device=device)
        self.observation_space = getattr(venv, "observation_space", None)
        self._frame = int(np.prod(self.frame_shape))

    def _stack(self, obs, done, reset):
        obs = obs.to(self.device, torch.float32).contiguous()
        if tuple(obs.shape) != (self.num_envs,) + self.frame_shape:
            raise ValueError("VecPyTorchFrameStack: obs shape %s, expected %s"
                             % (tuple(obs.shape), (self.num_envs,) + self.frame_shape))
        d = None
        if done is not None:
            d = torch.from_numpy(np.asarray(done, dtype=np.uint8)).to(self.device, non_blocking=True)
        call("ppo_frame_stack", self.stacked_obs.data_ptr(), self.num_envs, self.nstack, self._frame, obs.data_ptr(),
             None if d is None else d.data_ptr(), int(reset), stream())
        return self.stacked_obs

    def step_wait(self):
        obs, vector_obs, reward, done, info = self.venv.step_wait()
        return self._stack(obs, done, False), vector_obs, reward, done, info

    def step_async(self, actions):
        self.venv.step_async(actions)

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def reset(self):
        obs, vector_obs = self.venv.reset()
        return self._stack(obs, None, True), vector_obs

    def close(self):
        if hasattr(self.venv, "close"):
            self.venv.close()

    @property
    def vector_obs_len(self):
        return self.venv.vector_obs_len
