#!/usr/bin/env python3
"""Golden vectors for the observation boundary —
CONTAINER ONLY, never shipped to the GPU box.

Runs the reference's own wrapper classes from
/root/reference/ppo-dash-study/013_…/{sohojoe_wrappers,pytorch_wrappers}.py on
seeded u8 frames and records inputs + outputs into tests/golden/obs_boundary.npz:

  * NormalizeWrapper(env, "ObtRetro-v6") -> FrameStackMono(env, 2) -> TransposeImage
    -> VecPyTorch's .float(), the 013 "norm_obs" env chain (make_env.py:81-84),
    with the reference's own ObtRetro-v6_{mean,std}.txt (read as text);
  * the same with NormalizeWrapper(env) (u8 / 255) and with no normaliser (u8);
  * VecPyTorchFrameStack(venv, 4) over steps with dones.

gym, cv2 and baselines are not installed: minimal stand-ins provide the base
classes the wrappers subclass (gym.Wrapper, gym.ObservationWrapper, spaces.Box,
baselines VecEnvWrapper) and cv2.cvtColor(COLOR_RGB2GRAY) as OpenCV documents it
for float32 (R*0.299 + G*0.587 + B*0.114) — so the mono values are pinned only
to that formula ("parity unpinned" against cv2), while everything the
reference's code itself does (float64 normalisation, channel order, the
transposition of the mono plane, deque order, done-zeroing) is recorded from it.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden_obs.py
"""
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
import torch  # noqa: E402

REF = [os.path.join("/root/reference/ppo-dash-study", d) for d in sorted(os.listdir("/root/reference/ppo-dash-study"))
       if d.startswith("013_")][0]
NORM = [os.path.join("/root/reference/ppo-dash-study", d) for d in sorted(os.listdir("/root/reference/ppo-dash-study"))
        if d.startswith("011_")][0]
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "obs_boundary.npz")


def install_stubs():
    gym = types.ModuleType("gym")

    class Wrapper(object):
        def __init__(self, env):
            self.env = env
            self.observation_space = env.observation_space
            self.action_space = getattr(env, "action_space", None)

        def reset(self, **kw):
            return self.env.reset(**kw)

        def step(self, action):
            return self.env.step(action)

    class ObservationWrapper(Wrapper):
        def reset(self, **kw):
            return self.observation(self.env.reset(**kw))

        def step(self, action):
            ob, r, d, i = self.env.step(action)
            return self.observation(ob), r, d, i

    class Box(object):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.broadcast_to(np.asarray(low, dtype=np.float64), shape).copy()
            self.high = np.broadcast_to(np.asarray(high, dtype=np.float64), shape).copy()
            self.shape, self.dtype = shape, dtype

    spaces = types.ModuleType("gym.spaces")
    spaces.Box = Box
    spaces.Dict = dict
    spaces.Discrete = type("Discrete", (), {"__init__": lambda self, n: setattr(self, "n", n)})
    box_mod = types.ModuleType("gym.spaces.box")
    box_mod.Box = Box
    gym.Wrapper, gym.ObservationWrapper, gym.ActionWrapper = Wrapper, ObservationWrapper, Wrapper
    gym.spaces = spaces
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "gym.spaces.box": box_mod})

    cv2 = types.ModuleType("cv2")
    cv2.COLOR_RGB2GRAY = 7

    def cvtColor(img, code):   # OpenCV RGB2Gray<float>, left-to-right fp32
        assert code == 7 and img.dtype == np.float32
        return (img[..., 0] * np.float32(0.299) + img[..., 1] * np.float32(0.587)) + img[..., 2] * np.float32(0.114)

    cv2.cvtColor = cvtColor
    cv2.ocl = types.SimpleNamespace(setUseOpenCL=lambda flag: None)
    sys.modules["cv2"] = cv2

    for name in ("baselines", "baselines.common", "baselines.common.atari_wrappers", "baselines.common.vec_env",
                 "sohojoe_dummy_vec_env", "sohojoe_shmem_vec_env", "ppo", "ppo.envs"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["baselines.common.atari_wrappers"].LazyFrames = object

    class VecEnvWrapper(object):
        def __init__(self, venv, observation_space=None, action_space=None):
            self.venv = venv
            self.num_envs = venv.num_envs
            self.observation_space = observation_space or venv.observation_space

    sys.modules["baselines.common.vec_env"].VecEnvWrapper = VecEnvWrapper
    sys.modules["sohojoe_dummy_vec_env"].DummyVecEnv = object
    sys.modules["sohojoe_shmem_vec_env"].ShmemVecEnv = object
    sys.modules["ppo.envs"].VecNormalize = object
    return Box


class FrameEnv(object):
    """gym-style env replaying a fixed sequence of [84][84][3] u8 frames"""

    def __init__(self, frames, Box):
        self.frames, self.t = frames, 0
        self.observation_space = Box(0, 255, frames.shape[1:], np.uint8)
        self.observation_space.dtype = np.uint8

    def reset(self):
        self.t = 0
        return self.frames[0]

    def step(self, action):
        self.t += 1
        return self.frames[self.t], 0.0, False, {}


def main():
    Box = install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(NORM)   # NormalizeWrapper loads "ObtRetro-v6_{mean,std}.txt" relative to the cwd
    import sohojoe_wrappers as W
    import pytorch_wrappers as P
    rng = np.random.default_rng(2024)
    T, N = 3, 2
    frames = rng.integers(0, 256, size=(N, T, 84, 84, 3), dtype=np.uint8)
    outs = {}
    for tag, make in (("norm", lambda e: W.NormalizeWrapper(e, "ObtRetro-v6")),
                      ("div255", lambda e: W.NormalizeWrapper(e)),
                      ("raw", lambda e: e)):
        res = np.zeros((T, N, 4, 84, 84), np.float32)
        for n in range(N):
            env = P.TransposeImage(W.FrameStackMono(make(FrameEnv(frames[n], Box)), 2), op=[2, 0, 1])
            ob = env.reset()
            res[0, n] = torch.from_numpy(ob).float().numpy()   # VecPyTorch.reset (pytorch_wrappers.py:121-133)
            for t in range(1, T):
                ob, _, _, _ = env.step(0)
                res[t, n] = torch.from_numpy(ob).float().numpy()
        outs["out_" + tag] = res
    mean = np.loadtxt("ObtRetro-v6_mean.txt").reshape(84, 84, 3)
    std = np.loadtxt("ObtRetro-v6_std.txt")
    os.chdir(cwd)

    # VecPyTorchFrameStack(venv, 4) over 6 steps with dones
    NS, NE, SH = 4, 3, (3, 10, 10)
    seq = rng.random((7, NE) + SH, dtype=np.float32)
    dones = rng.random((7, NE)) < 0.35

    class VEnv(object):
        num_envs = NE
        observation_space = Box(0.0, 1.0, SH)

        def __init__(self):
            self.t = 0

        def reset(self):
            self.t = 0
            return torch.from_numpy(seq[0]), torch.zeros(0)

        def step_wait(self):
            self.t += 1
            return torch.from_numpy(seq[self.t]), torch.zeros(0), None, dones[self.t], {}

    fs = P.VecPyTorchFrameStack(VEnv(), NS, torch.device("cpu"))
    st = [fs.reset()[0].clone().numpy()]
    for _ in range(6):
        st.append(fs.step_wait()[0].clone().numpy())
    np.savez_compressed(OUT, frames=frames, mean=mean, std=np.float64(std), **outs, fs_seq=seq, fs_dones=dones,
                        fs_stacked=np.stack(st), fs_nstack=np.int64(NS))
    print("wrote", OUT, {k: v.shape for k, v in outs.items()})


if __name__ == "__main__":
    main()
