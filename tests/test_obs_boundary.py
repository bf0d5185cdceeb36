"""Observation boundary: the reference's env-side chain
NormalizeWrapper -> FrameStackMono(2) -> TransposeImage -> VecPyTorch .float()
and VecPyTorchFrameStack, against golden vectors recorded from the reference's
own wrapper classes (tools/gen_golden_obs.py).  Bit-exact throughout; the grey
plane follows OpenCV's published RGB2GRAY formula (cv2 itself is not installed:
that plane is parity-unpinned against cv2)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import obs_oracle as O

MODES = ("norm", "div255", "raw")


def _same(got, ref, what):
    """bit-exact comparison with a short failure message"""
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    bad = got.view(np.uint32) != ref.view(np.uint32) if got.dtype == np.float32 else got != ref
    if bad.any():
        idx = np.argwhere(bad)[:4].tolist()
        raise AssertionError("%s: %d of %d elements differ, first at %s" % (what, int(bad.sum()), bad.size, idx))


def _oracle_args(g, mode):
    if mode == "norm":
        return dict(mean=g["mean"], std=g["std"])
    return dict(div255=(mode == "div255"))


@pytest.mark.parametrize("mode", MODES)
def test_oracle_matches_reference_chain(mode):
    g = golden("obs_boundary.npz")
    frames, ref = g["frames"], g["out_" + mode]   # frames [N][T][84][84][3], ref [T][N][4][84][84]
    T = frames.shape[1]
    for t in range(T):
        got = O.preprocess_batch(frames[:, t], **_oracle_args(g, mode))
        assert np.array_equal(got, ref[t]), (mode, t)


def test_oracle_frame_stack_matches_reference():
    g = golden("obs_boundary.npz")
    seq, dones, ref = g["fs_seq"], g["fs_dones"], g["fs_stacked"]
    fs = O.VecFrameStack(seq.shape[1], int(g["fs_nstack"]), seq.shape[2:])
    got = [fs.reset(seq[0])] + [fs.step(seq[t], dones[t]) for t in range(1, seq.shape[0])]
    assert np.array_equal(np.stack(got), ref)


def test_mono_plane_is_transposed_in_the_reference():
    """the reference stacks (W,H) colour planes with an (H,W) grey image, so its
    grey channel at (y, x) is gray(frame[x][y]); the golden file shows it"""
    g = golden("obs_boundary.npz")
    f = g["frames"][0, 0]
    gray = O.gray_f32(f.astype(np.float64))
    assert np.array_equal(g["out_raw"][0, 0, 3], gray.astype(np.uint8).T.astype(np.float32))
    assert not np.array_equal(g["out_raw"][0, 0, 3], gray.astype(np.uint8).astype(np.float32))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_obs_preprocess_kernel_golden(gpu, mode):
    from a2c_ppo_acktr.vec_env import ObsPreprocess
    g = golden("obs_boundary.npz")
    frames, ref = g["frames"], g["out_" + mode]
    pre = ObsPreprocess(84, mode, g["mean"] if mode == "norm" else None, g["std"] if mode == "norm" else None,
                        device=gpu)
    for t in range(frames.shape[1]):
        out = pre(torch.from_numpy(np.ascontiguousarray(frames[:, t])).to(gpu))
        torch.cuda.synchronize()
        _same(out.cpu().numpy(), ref[t], (mode, t))


@pytest.mark.gpu
def test_obs_preprocess_into_storage_slot_and_edge_cases(gpu):
    """writes straight into a strided fp32 storage slot; N=0 is a no-op; wrong
    shapes raise; a large random batch matches the oracle bit for bit"""
    from a2c_ppo_acktr.vec_env import ObsPreprocess
    g = golden("obs_boundary.npz")
    pre = ObsPreprocess(84, "norm", g["mean"], g["std"], device=gpu)
    rng = np.random.default_rng(5)
    N = 37
    fr = rng.integers(0, 256, size=(N, 84, 84, 3), dtype=np.uint8)
    obs = torch.full((3, N, 4, 84, 84), float("nan"), device=gpu)   # a [T+1][N][C][H][W] storage plane
    pre(torch.from_numpy(fr).to(gpu), out=obs[1])
    torch.cuda.synchronize()
    _same(obs[1].cpu().numpy(), O.preprocess_batch(fr, mean=g["mean"], std=g["std"]), "slot")
    assert torch.isnan(obs[0]).all() and torch.isnan(obs[2]).all()
    empty = pre(torch.zeros(0, 84, 84, 3, dtype=torch.uint8, device=gpu))
    assert empty.shape == (0, 4, 84, 84)
    with pytest.raises(TypeError):
        pre(torch.zeros(2, 84, 84, 4, dtype=torch.uint8, device=gpu))
    with pytest.raises(TypeError):
        pre(torch.zeros(2, 84, 84, 3, dtype=torch.float32, device=gpu))


@pytest.mark.gpu
def test_frame_stack_kernel_golden(gpu):
    from a2c_ppo_acktr.vec_env import VecPyTorchFrameStack
    g = golden("obs_boundary.npz")
    seq, dones, ref = g["fs_seq"], g["fs_dones"], g["fs_stacked"]

    class Box:
        shape = seq.shape[2:]

    class VEnv:
        num_envs = seq.shape[1]
        observation_space = Box()
        vector_obs_len = 0
        t = 0

        def reset(self):
            self.t = 0
            return torch.from_numpy(seq[0]).to(gpu), None

        def step_wait(self):
            self.t += 1
            return torch.from_numpy(seq[self.t]).to(gpu), None, None, dones[self.t], {}

    fs = VecPyTorchFrameStack(VEnv(), int(g["fs_nstack"]), gpu)
    got = [fs.reset()[0].cpu().numpy()]
    for _ in range(seq.shape[0] - 1):
        got.append(fs.step_wait()[0].cpu().numpy())
    _same(np.stack(got), ref, "frame stack")


@pytest.mark.gpu
def test_vec_pytorch_end_to_end(gpu):
    """VecPyTorch over a host vec env that returns raw u8 RGB frames + vector obs
    (dict spaces, as the OTC env): u8 crosses PCIe, the device chain reproduces
    the reference's per-env wrappers; rewards come back [N,1] on the host"""
    from a2c_ppo_acktr.vec_env import ObsPreprocess, VecPyTorch
    g = golden("obs_boundary.npz")
    frames = g["frames"]                      # [N][T][84][84][3]
    N, T = frames.shape[:2]

    class Space:
        def __init__(self, shape):
            self.shape = shape

    class HostVecEnv:
        num_envs = N
        observation_space = type("D", (), {"spaces": {"visual": Space((84, 84, 3)), "vector": Space((14,))}})()

        def __init__(self):
            self.t = 0

        def _obs(self):
            return {"visual": frames[:, self.t].copy(), "vector": np.full((N, 14), self.t, np.float32)}

        def reset(self):
            self.t = 0
            return self._obs()

        def step_async(self, a):
            self.actions = a

        def step_wait(self):
            self.t += 1
            return self._obs(), np.arange(N, dtype=np.float32), np.zeros(N, bool), [{}] * N

    env = VecPyTorch(HostVecEnv(), gpu, preprocess=ObsPreprocess(84, "norm", g["mean"], g["std"], device=gpu))
    assert env.vector_obs_len == 14
    vis, vec = env.reset()
    outs = [vis.cpu().numpy()]
    for t in range(1, T):
        vis, vec, rew, done, info = env.step(torch.zeros(N, 1, dtype=torch.int64, device=gpu))
        assert rew.shape == (N, 1) and vec.shape == (N, 14) and vec.device == gpu and float(vec[0, 0]) == t
        outs.append(vis.cpu().numpy())
    _same(np.stack(outs), g["out_norm"], "VecPyTorch")
