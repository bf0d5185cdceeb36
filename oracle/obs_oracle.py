"""ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker (or the timed CPU baseline).  The product
path (ppo-dash_amd/) never imports it.

A numpy restatement of the observation boundary, paths
relative to ppo-dash-study/013_ra+no_stack+lshp+recurrent+vec_obs+norm_obs+rew_hacking/:

  * NormalizeWrapper.observation     sohojoe_wrappers.py:872-884  -> normalize()
  * FrameStackMono(k)._add_ob/_get_ob sohojoe_wrappers.py:425-501 -> FrameStackMono
  * TransposeImage (op [2, 0, 1])    pytorch_wrappers.py:170-203  -> np.transpose
  * VecPyTorch.step_wait .float()    pytorch_wrappers.py:105-160  -> astype(float32)
  * VecPyTorchFrameStack             pytorch_wrappers.py:58-102   -> VecFrameStack

cv2 is not installed here, so cv2.cvtColor(COLOR_RGB2GRAY) on float32 is
restated from OpenCV's published RGB2Gray<float> (R·0.299 + G·0.587 + B·0.114,
fp32, left to right): that channel is "parity unpinned" against cv2 itself.
Everything else (float64 normalisation, channel order, the transposed mono
plane, deque order, done-zeroing) is pinned by tests/golden/obs_boundary.npz,
recorded by running the reference's own wrapper classes (tools/gen_golden_obs.py).
"""
from collections import deque

import numpy as np


def gray_f32(img):
    """cv2.cvtColor(img.astype(float32), COLOR_RGB2GRAY) for an [H][W][3] image"""
    x = img.astype(np.float32)
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    return (r * np.float32(0.299) + g * np.float32(0.587)) + b * np.float32(0.114)


def normalize(frame_u8, mean=None, std=None, div255=True):
    """NormalizeWrapper.observation (013 copy, `is not None` test): float64"""
    if mean is not None:
        return (frame_u8 - mean) / std
    if div255:
        return frame_u8 / 255
    return frame_u8


class FrameStackMono(object):
    """_add_ob / _get_ob of FrameStackMono(k): colour planes of the newest frame +
    mono_frames[1..k-1]; np.array(list(frames)).T as the reference builds it."""

    def __init__(self, k):
        self.k = k
        self.frames = deque([], maxlen=3 + (k - 1))
        self.color_frames = deque([], maxlen=3)
        self.mono_frames = deque([], maxlen=k)

    def _add_ob(self, ob):
        ob_t = ob.T
        for c in range(3):
            self.color_frames.append(ob_t[c])
        self.mono_frames.append(gray_f32(ob).astype(ob.dtype))

    def _get_ob(self):
        for c in range(3):
            self.frames.append(self.color_frames[c])
        for i in range(self.k - 1):
            self.frames.append(self.mono_frames[i + 1])
        return np.array(list(self.frames)).T

    def reset(self, ob):
        for _ in range(self.k):
            self._add_ob(ob)
        return self._get_ob()

    def step(self, ob):
        self._add_ob(ob)
        return self._get_ob()


def policy_input(hwc):
    """TransposeImage [2, 0, 1] then VecPyTorch's .float()"""
    return np.ascontiguousarray(np.transpose(hwc, (2, 0, 1))).astype(np.float32)


class VecFrameStack(object):
    """VecPyTorchFrameStack on numpy: stacked [N][nstack*C][H][W] fp32"""

    def __init__(self, num_envs, nstack, frame_shape):
        self.C = frame_shape[0]
        self.stacked = np.zeros((num_envs, nstack * self.C) + tuple(frame_shape[1:]), np.float32)

    def reset(self, obs):
        self.stacked[...] = 0
        self.stacked[:, -self.C:] = obs
        return self.stacked.copy()

    def step(self, obs, done):
        self.stacked[:, :-self.C] = self.stacked[:, self.C:]
        for i, new in enumerate(done):
            if new:
                self.stacked[i] = 0
        self.stacked[:, -self.C:] = obs
        return self.stacked.copy()


def preprocess_batch(frames_u8, mean=None, std=None, div255=True, mono=True):
    """One step of N independent envs right after a reset (FrameStackMono state =
    this frame): [N][S][S][3] u8 -> [N][3 (+1)][S][S] fp32 policy input."""
    out = []
    for f in frames_u8:
        x = normalize(f, mean, std, div255)
        if mono:
            x = FrameStackMono(2).reset(x)
        out.append(policy_input(x))
    return np.stack(out)
