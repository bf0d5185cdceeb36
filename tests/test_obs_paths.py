"""conv1 on the observation forms of the reference's own env chain (GPU;
csrc/conv1f.hip):

  * fp32 rows [4][84][84] — the fp32 storage plane T/run.py fills unchanged
    (T/a2c_ppo_acktr/storage.py:12, T/make_env.py:96-114);
  * raw u8 RGB frames [84][84][3] decoded in conv1's loader as NormalizeWrapper +
    FrameStackMono(2) + TransposeImage + .float() (T/make_env.py:411-413).

Checks: the fused decode reproduces the reference chain BIT-EXACTLY (read back
through selector weights, against oracle/obs_oracle.py, itself pinned to
tests/golden/obs_boundary.npz recorded from the reference's wrapper classes);
forward / ReLU mask bits / weight + bias gradients vs torch float64 at 1e-5 of
max|ref| (the bar of the u8 kernels' tests); full c3 minibatch gradients live in
test_full_size.py."""
import numpy as np
import pytest
import torch

from oracle import obs_oracle as OO

pytestmark = pytest.mark.gpu


def _hip():
    from a2c_ppo_acktr import _hip
    return _hip


def _s():
    return torch.cuda.current_stream().cuda_stream


def _mean(seed=0):
    """a NormalizeWrapper mean file's shape and value range, fp32-representable as
    ObtRetro-v6_mean.txt's values are"""
    return np.random.default_rng(seed).uniform(20, 80, (84, 84, 3)).astype(np.float32).astype(np.float64)


MODES = {"norm": (lambda: _mean(), 36.31282043457031), "div255": (lambda: None, 255.0), "raw": (lambda: None, 1.0)}


def _decoded(frames, mode):
    """the reference chain on the host: [N][84][84][3] u8 -> [N][4][84][84] fp32"""
    mean, std = MODES[mode][0](), MODES[mode][1]
    if mode == "norm":
        return OO.preprocess_batch(frames, mean=mean, std=std), mean, std
    return OO.preprocess_batch(frames, div255=(mode == "div255")), None, std


def _fwd(src, obs_d, idx_d, B, w, b, mbits=None, mean=None, std=1.0):
    H = _hip()
    out = torch.empty(B, 20, 20, 32, device="cuda")
    if src == "f32":
        H.call("ppo_conv1_fwd_f32", obs_d.data_ptr(), None if idx_d is None else idx_d.data_ptr(), 0, B,
               w.data_ptr(), b.data_ptr(), out.data_ptr(), None if mbits is None else mbits.data_ptr(), _s())
    else:
        H.call("ppo_conv1_fwd_rgb", obs_d.data_ptr(), None if idx_d is None else idx_d.data_ptr(), 0, B,
               None if mean is None else mean.data_ptr(), std, w.data_ptr(), b.data_ptr(), out.data_ptr(),
               None if mbits is None else mbits.data_ptr(), _s())
    return out


@pytest.mark.parametrize("src", ["rgb", "f32"])
@pytest.mark.parametrize("mode", ["norm", "div255", "raw"])
def test_fused_decode_bit_exact(gpu, mode, src):
    """Selector weights (+1 / -1 on one tap per output channel, zero bias) make
    conv1's output relu(±x) of single input elements; with exact unit weights the
    six split products sum back to x itself, so the decoded inputs are read back
    exactly: every element of the 80x80 tap window of all four channels (colour
    planes and the transposed grey plane) equals the reference chain's bit for bit.
    (The fused-decode kernel, rgb_aff 0; the affine fold, test_rgb_affine_*, forms
    no per-element fl32 of the decode and is checked against float64 instead.)"""
    H = _hip()
    old_aff = H.call("ppo_tune_get", b"rgb_aff")
    H.call("ppo_tune_set", b"rgb_aff", 0)
    try:
        _decode_readback(gpu, mode, src)
    finally:
        H.call("ppo_tune_set", b"rgb_aff", old_aff)


def _decode_readback(gpu, mode, src):
    g = torch.Generator().manual_seed(11)
    N = 6
    frames = torch.randint(0, 256, (N, 84, 84, 3), dtype=torch.uint8, generator=g)
    frames[0] = 0
    frames[1] = 255
    ref, mean, std = _decoded(frames.numpy(), mode)
    fr_d = frames.cuda()
    mean_d = None if mean is None else torch.from_numpy(mean.astype(np.float32)).cuda()
    got = np.zeros((N, 4, 80, 80), np.float32)
    for c in range(4):
        w = torch.zeros(32, 4, 8, 8)
        for ky in range(4):
            for kx in range(4):
                w[ky * 4 + kx, c, ky, kx] = 1.0
                w[16 + ky * 4 + kx, c, ky, kx] = -1.0
        if src == "rgb":
            out = _fwd("rgb", fr_d, None, N, w.cuda().contiguous(), torch.zeros(32, device=gpu), mean=mean_d,
                       std=std).cpu().numpy()
        else:   # the reference chain's fp32 values through the fp32-input kernel
            out = _fwd("f32", torch.from_numpy(ref).cuda(), None, N, w.cuda().contiguous(),
                       torch.zeros(32, device=gpu)).cpu().numpy()
        for ky in range(4):
            for kx in range(4):
                pos, neg = out[..., ky * 4 + kx], out[..., 16 + ky * 4 + kx]
                got[:, c, ky::4, kx::4] = pos - neg   # one of them is 0
    bad = got != ref[:, :, :80, :80]
    print(src, mode, "mismatches per channel", bad.sum((0, 2, 3)), "per (ky, kx)",
          bad.reshape(N, 4, 20, 4, 20, 4).sum((0, 1, 2, 4)).tolist())
    if bad.any():
        i = np.argwhere(bad)[0]
        r = ref[tuple(i[:2]) + (i[2], i[3])]
        print("first", i, got[tuple(i)], r, np.float32(got[tuple(i)]).view(np.uint32), np.float32(r).view(np.uint32))
    np.testing.assert_array_equal(got, ref[:, :, :80, :80])


def test_rgb_affine_raw_mode_keeps_decode(gpu):
    """The raw mode (no normaliser, s = 1) stores FrameStackMono's grey plane as
    truncated u8 — not affine in the bytes — so with the affine fold on it must
    still take the fused decode: the bit-exact read-back holds."""
    H = _hip()
    old_aff = H.call("ppo_tune_get", b"rgb_aff")
    H.call("ppo_tune_set", b"rgb_aff", 1)
    try:
        _decode_readback(gpu, "raw", "rgb")
    finally:
        H.call("ppo_tune_set", b"rgb_aff", old_aff)


@pytest.mark.parametrize("mode", ["norm", "div255"])
def test_rgb_affine_vs_float64(gpu, mode):
    """The affine fold (rgbaff.hip) in both affine modes, whole frames (idx None),
    B = 5 < the grid, extreme frames (all 0, all 255) included: forward + ReLU vs
    torch float64 of the reference chain's decoded input at 1e-5 of max|ref|."""
    H = _hip()
    g = torch.Generator().manual_seed(23)
    B = 5
    frames = torch.randint(0, 256, (B, 84, 84, 3), dtype=torch.uint8, generator=g)
    frames[0] = 0
    frames[1] = 255
    dec, mean, std = _decoded(frames.numpy(), mode)
    w = torch.randn(32, 4, 8, 8, generator=g) * 0.05
    b = torch.randn(32, generator=g) * 0.1
    mean_d = None if mean is None else torch.from_numpy(mean.astype(np.float32)).cuda()
    old_aff = H.call("ppo_tune_get", b"rgb_aff")
    H.call("ppo_tune_set", b"rgb_aff", 1)
    try:
        out = _fwd("rgb", frames.cuda(), None, B, w.cuda(), b.cuda(), None, mean_d, std)
        torch.cuda.synchronize()
    finally:
        H.call("ppo_tune_set", b"rgb_aff", old_aff)
    ref = torch.relu(torch.nn.functional.conv2d(torch.from_numpy(dec).double(), w.double(), b.double(),
                                                stride=4)).permute(0, 2, 3, 1)
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


@pytest.mark.parametrize("src", ["f32", "rgb", "rgb_decode"])
@pytest.mark.parametrize("products", [6, 9, 1])
def test_conv1_fwd_vs_float64(gpu, src, products):
    """forward + bias + ReLU and the ReLU mask bits, rows gathered out of order,
    B = 300 > the persistent grid (blocks walk several images): 1e-5 of max|ref|
    (products 6 / 9: fp32 accuracy), bf16 operand rounding (1: half-precision mode).
    rgb: the affine fold (rgbaff.hip, default); rgb_decode: the fused decode."""
    H = _hip()
    old_aff = H.call("ppo_tune_get", b"rgb_aff")
    H.call("ppo_tune_set", b"rgb_aff", 0 if src == "rgb_decode" else 1)
    try:
        _fwd_vs_float64(gpu, "rgb" if src == "rgb_decode" else src, products)
    finally:
        H.call("ppo_tune_set", b"rgb_aff", old_aff)


def _fwd_vs_float64(gpu, src, products):
    H = _hip()
    g = torch.Generator().manual_seed(5 + products)
    B, rows = 300, 420
    idx = torch.randperm(rows, generator=g)[:B].contiguous()
    w = torch.randn(32, 4, 8, 8, generator=g) * 0.05
    b = torch.randn(32, generator=g) * 0.1
    if src == "f32":
        obs = torch.randn(rows, 4, 84, 84, generator=g)
        x = obs[idx].double()
        obs_d, mean_d, std = obs.cuda(), None, 1.0
    else:
        frames = torch.randint(0, 256, (rows, 84, 84, 3), dtype=torch.uint8, generator=g)
        dec, mean, std = _decoded(frames[idx].numpy(), "norm")
        x = torch.from_numpy(dec).double()
        obs_d, mean_d = frames.cuda(), torch.from_numpy(mean.astype(np.float32)).cuda()
    mbits = torch.zeros(B * 400, dtype=torch.int32, device=gpu)
    old = H.call("ppo_tune_get", b"products")
    H.call("ppo_tune_set", b"products", products)
    try:
        out = _fwd(src, obs_d, idx.cuda(), B, w.cuda(), b.cuda(), mbits, mean_d, std)
        torch.cuda.synchronize()
    finally:
        H.call("ppo_tune_set", b"products", old)
    ref = torch.relu(torch.nn.functional.conv2d(x, w.double(), b.double(), stride=4)).permute(0, 2, 3, 1)
    got = out.cpu().double()
    tol = 1e-5 if products != 1 else 2e-2
    err = (got - ref).abs().max().item()
    assert err <= tol * ref.abs().max().item(), err
    bits = mbits.cpu().numpy().view(np.uint32).reshape(B, 400)
    want = (out.cpu().numpy().reshape(B, 400, 32) > 0)
    got_bits = ((bits[..., None] >> np.arange(32, dtype=np.uint32)) & 1).astype(bool)
    assert np.array_equal(got_bits, want)


@pytest.mark.parametrize("src", ["f32", "rgb", "rgb_decode", "rgb_few"])
@pytest.mark.parametrize("products", [6, 9])
def test_conv1_wgrad_vs_float64(gpu, src, products):
    """weight + bias gradient, rows gathered out of order, B = 300 over a Z that
    leaves blocks with one and with two images: 1e-5 of max|ref|.  rgb: the affine
    fold (two passes + the means' share, rgbaff.hip), rgb_few: the same with B = 100
    < Z (blocks without images), rgb_decode: the fused-decode kernel."""
    H = _hip()
    old_aff = H.call("ppo_tune_get", b"rgb_aff")
    H.call("ppo_tune_set", b"rgb_aff", 0 if src == "rgb_decode" else 1)
    try:
        _wgrad_vs_float64(gpu, "f32" if src == "f32" else "rgb", products, 100 if src == "rgb_few" else 300)
    finally:
        H.call("ppo_tune_set", b"rgb_aff", old_aff)


def _wgrad_vs_float64(gpu, src, products, B):
    H = _hip()
    g = torch.Generator().manual_seed(17 + products)
    rows = 420
    idx = torch.randperm(rows, generator=g)[:B].contiguous()
    dz1 = torch.randn(B, 20, 20, 32, generator=g)
    if src == "f32":
        obs = torch.randn(rows, 4, 84, 84, generator=g)
        x = obs[idx].double()
        obs_d, mean_d, std = obs.cuda(), None, 1.0
    else:
        frames = torch.randint(0, 256, (rows, 84, 84, 3), dtype=torch.uint8, generator=g)
        dec, mean, std = _decoded(frames[idx].numpy(), "norm")
        x = torch.from_numpy(dec).double()
        obs_d, mean_d = frames.cuda(), torch.from_numpy(mean.astype(np.float32)).cuda()
    Z = 256
    slab = torch.empty(Z * 32 * 256, device=gpu)
    slab_b = torch.empty(Z * 32, device=gpu)
    gw = torch.empty(32 * 256, device=gpu)
    gb = torch.empty(32, device=gpu)
    dz1_d, idx_d = dz1.cuda(), idx.cuda()
    old = H.call("ppo_tune_get", b"products")
    H.call("ppo_tune_set", b"products", products)
    try:
        if src == "f32":
            H.call("ppo_conv1_wgrad_f32", dz1_d.data_ptr(), obs_d.data_ptr(), idx_d.data_ptr(), 0, B, Z,
                   slab.data_ptr(), slab_b.data_ptr(), _s())
        else:
            H.call("ppo_conv1_wgrad_rgb", dz1_d.data_ptr(), obs_d.data_ptr(), idx_d.data_ptr(), 0, B,
                   mean_d.data_ptr(), std, Z, slab.data_ptr(), slab_b.data_ptr(), _s())
        H.call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, 32, 256, 0, 0, 0, gw.data_ptr(),
               gb.data_ptr(), 1.0, 0, _s())
        torch.cuda.synchronize()
    finally:
        H.call("ppo_tune_set", b"products", old)
    dy = dz1.double().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(x, (32, 4, 8, 8), dy, stride=4)
    ref_b = dy.sum((0, 2, 3))
    for got, ref in ((gw.cpu().double().view(32, 4, 8, 8), ref_w), (gb.cpu().double(), ref_b)):
        err = (got - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item(), err


def test_engine_routes_float_obs_to_image_resident_kernel(gpu):
    """ppo_conv1_fwd / ppo_conv1_wgrad with fp32 observations (C = 4) take the
    conv1f.hip kernels: same results as calling them directly (bit-identical)."""
    H = _hip()
    g = torch.Generator().manual_seed(3)
    B = 40
    obs = torch.randn(B, 4, 84, 84, generator=g).cuda()
    w = (torch.randn(32, 4, 8, 8, generator=g) * 0.05).cuda()
    b = torch.zeros(32).cuda()
    a = torch.empty(B, 20, 20, 32, device=gpu)
    H.call("ppo_conv1_fwd", obs.data_ptr(), 0, None, 0, 4, B, w.data_ptr(), b.data_ptr(), a.data_ptr(), _s())
    ref = _fwd("f32", obs, None, B, w, b)
    torch.cuda.synchronize()
    assert torch.equal(a, ref)
