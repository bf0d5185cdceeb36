"""CNNBase fc GEMMs (GPU): the split-bf16 tile kernels (igemm_x9.h: the fc
forward and dgrad split in the k loop, the weight gradient split at staging;
ppo_tune_set("x9", 1), default) and the fp32-MFMA tile core (x9 0), through the
C ABI, vs torch float64 — the fc forward (model.py:181, Linear(32*7*7, H) + ReLU)
and its input gradient masked by conv3's ReLU (threshold_backward of the
flatten/ReLU in CNNBase.main).  Bar: 1e-5 of max|ref| with the fp32-accurate
split (6 / 9 products), bf16-operand rounding (2e-2) in half-precision mode (1)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    from a2c_ppo_acktr import _hip
    return _hip


def _s():
    return torch.cuda.current_stream().cuda_stream


def _packed(gpu, H, seed):
    H_ = _hip()
    g = torch.Generator().manual_seed(seed)
    w2 = torch.randn(64, 32, 4, 4, generator=g) * 0.05
    w3 = torch.randn(32, 64, 3, 3, generator=g) * 0.05
    w4 = torch.randn(H, 1568, generator=g) * 0.03
    packed = torch.empty(H_.call("ppo_packed_weights_size", H), device=gpu)
    offs = torch.zeros(6, dtype=torch.int64)
    H_.call("ppo_packed_offsets", H, offs.data_ptr())
    d = [t.cuda() for t in (w2, w3, w4)]
    H_.call("ppo_pack_weights", d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), H, packed.data_ptr(), _s())
    pk = [packed.data_ptr() + 4 * int(o) for o in offs]
    # the packed fc weight's columns follow the engine's HWC activation layout
    # ([B][7][7][32]); torch's flatten is CHW
    return w4.view(H, 32, 7, 7).permute(0, 2, 3, 1).reshape(H, 1568), packed, pk


def _with_tune(key, value, products, fn):
    H_ = _hip()
    old, oldp = H_.call("ppo_tune_get", key), H_.call("ppo_tune_get", b"products")
    H_.call("ppo_tune_set", key, value)
    H_.call("ppo_tune_set", b"products", products)
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        H_.call("ppo_tune_set", key, old)
        H_.call("ppo_tune_set", b"products", oldp)


@pytest.mark.parametrize("x9", [1, 0])
@pytest.mark.parametrize("products", [6, 9, 1])
@pytest.mark.parametrize("B,H", [(300, 512), (77, 64), (129, 256), (4096, 512)])
def test_fc_fwd_vs_float64(gpu, x9, products, B, H):
    """relu(x W^T + b) with B not a multiple of the 128-row tile and H = 64 (waves
    without weight rows), written into a wider output (ldo = H + 8)."""
    H_ = _hip()
    w4, packed, pk = _packed(gpu, H, 3 + H)
    g = torch.Generator().manual_seed(B)
    x = torch.relu(torch.randn(B, 1568, generator=g))
    b = torch.randn(H, generator=g) * 0.1
    ldo = H + 8
    out = torch.full((B, ldo), float("nan"), device=gpu)
    xd, bd = x.cuda(), b.cuda()
    _with_tune(b"x9", x9, products,
               lambda: H_.call("ppo_fc_fwd", xd.data_ptr(), B, pk[2], bd.data_ptr(), H, out.data_ptr(), ldo, _s()))
    ref = torch.relu(x.double() @ w4.double().t() + b.double())
    got = out[:, :H].cpu().double()
    tol = 1e-5 if products != 1 else 2e-2
    err = (got - ref).abs().max().item()
    assert err <= tol * ref.abs().max().item(), err
    assert torch.isnan(out[:, H:]).all()   # the padding columns are untouched


@pytest.mark.parametrize("x9", [1, 0])
@pytest.mark.parametrize("products", [6, 9, 1])
@pytest.mark.parametrize("B,H", [(300, 512), (77, 64), (200, 40)])
def test_fc_dgrad_mask_vs_float64(gpu, x9, products, B, H):
    """dx = [a3 > 0] * (dh W): N = 1568 = 6 full 256-row weight blocks + 32 rows;
    H = 40 ends the reduction inside a 32-wide k-step."""
    H_ = _hip()
    w4, packed, pk = _packed(gpu, H, 5 + H)
    g = torch.Generator().manual_seed(B + 1)
    dh = torch.randn(B, H, generator=g)
    a3 = torch.relu(torch.randn(B, 1568, generator=g))
    dx = torch.full((B, 1568), float("nan"), device=gpu)
    dhd, a3d = dh.cuda(), a3.cuda()
    _with_tune(b"x9", x9, products,
               lambda: H_.call("ppo_linear_dgrad_mask", dhd.data_ptr(), B, H, pk[3], 1568, a3d.data_ptr(),
                               dx.data_ptr(), _s()))
    ref = (dh.double() @ w4.double()) * (a3 > 0).double()
    got = dx.cpu().double()
    tol = 1e-5 if products != 1 else 2e-2
    err = (got - ref).abs().max().item()
    assert err <= tol * ref.abs().max().item(), err
    assert (got[a3 <= 0] == 0).all()


@pytest.mark.parametrize("x9", [1, 0])
@pytest.mark.parametrize("products", [6, 1])
@pytest.mark.parametrize("R,H", [(1000, 512), (333, 256)])
def test_fc_wgrad_vs_float64(gpu, x9, products, R, H):
    """dW[n][k] = Σ_r dh[r][n] a3[r][k] and db[n] = Σ_r dh[r][n] (the fc layer's
    weight gradient, model.py:181 under loss.backward()): split-K slabs over the
    rows, reduced in a fixed order; R not a multiple of the 32-row k-step."""
    H_ = _hip()
    g = torch.Generator().manual_seed(R + H)
    dh = torch.randn(R, H, generator=g)
    a3 = torch.relu(torch.randn(R, 1568, generator=g))
    Z = 7
    slab = torch.full((Z * H * 1568,), float("nan"), device=gpu)
    slab_b = torch.full((Z * H,), float("nan"), device=gpu)
    dhd, a3d = dh.cuda(), a3.cuda()
    _with_tune(b"x9", x9, products,
               lambda: H_.call("ppo_linear_wgrad", dhd.data_ptr(), a3d.data_ptr(), R, H, 1568, Z, slab.data_ptr(),
                               slab_b.data_ptr(), _s()))
    gw = slab.view(Z, H, 1568).sum(0).cpu().double()
    gb = slab_b.view(Z, H).sum(0).cpu().double()
    ref_w = dh.double().t() @ a3.double()
    ref_b = dh.double().sum(0)
    tol = 1e-5 if products != 1 else 2e-2
    assert (gw - ref_w).abs().max().item() <= tol * ref_w.abs().max().item()
    assert (gb - ref_b).abs().max().item() <= 1e-5 * ref_b.abs().max().item()


@pytest.mark.parametrize("Z", [2, 3, 4])
@pytest.mark.parametrize("B,H", [(4096, 512), (1000, 256), (77, 64)])
def test_fc_fwd_splitk_vs_float64(gpu, Z, B, H):
    """ppo_fc_fwd_ws: the rollout-sized split-K fc forward (Z K-slices into the
    workspace, fixed-order reduce + bias + ReLU) vs torch float64, and vs the
    unsplit kernel within fp32 summation-order noise; a short workspace falls back."""
    H_ = _hip()
    w4, packed, pk = _packed(gpu, H, 7 + H)
    g = torch.Generator().manual_seed(B + Z)
    x = torch.relu(torch.randn(B, 1568, generator=g))
    b = torch.randn(H, generator=g) * 0.1
    xd, bd = x.cuda(), b.cuda()
    old = H_.call("ppo_tune_get", b"fc_splitk")
    H_.call("ppo_tune_set", b"fc_splitk", Z)
    try:
        nb = H_.call("ppo_fc_fwd_ws_bytes", B, H)
        assert nb == 4 * Z * B * H
        ws = torch.full((nb // 4,), float("nan"), device=gpu)
        out = torch.full((B, H), float("nan"), device=gpu)
        H_.call("ppo_fc_fwd_ws", xd.data_ptr(), B, pk[2], bd.data_ptr(), H, out.data_ptr(), H, ws.data_ptr(), nb, _s())
        ref_ub = torch.empty(B, H, device=gpu)
        H_.call("ppo_fc_fwd", xd.data_ptr(), B, pk[2], bd.data_ptr(), H, ref_ub.data_ptr(), H, _s())
        short = torch.empty(B, H, device=gpu)
        H_.call("ppo_fc_fwd_ws", xd.data_ptr(), B, pk[2], bd.data_ptr(), H, short.data_ptr(), H, ws.data_ptr(), nb - 4,
                _s())
        torch.cuda.synchronize()
    finally:
        H_.call("ppo_tune_set", b"fc_splitk", old)
    ref = torch.relu(x.double() @ w4.double().t() + b.double())
    got = out.cpu().double()
    assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    assert (got - ref_ub.cpu().double()).abs().max().item() <= 2e-6 * ref.abs().max().item()
    assert torch.equal(short, ref_ub)   # too small a workspace: the unsplit kernel


@pytest.mark.parametrize("Z", [2, 3])
@pytest.mark.parametrize("B,H", [(4096, 512), (1000, 256), (77, 64)])
def test_fc_splitk_tiles_bit_identical(gpu, Z, B, H):
    """fc_splitk_tile 1 (128 x 128 tiles, 16-B slab stores) and 0 (128 x 64) run the same
    k order and part products per output: bit-identical outputs"""
    H_ = _hip()
    w4, packed, pk = _packed(gpu, H, 9 + H)
    g = torch.Generator().manual_seed(B + 3 * Z)
    xd = torch.relu(torch.randn(B, 1568, generator=g)).cuda()
    bd = (torch.randn(H, generator=g) * 0.1).cuda()
    old = H_.call("ppo_tune_get", b"fc_splitk"), H_.call("ppo_tune_get", b"fc_splitk_tile")
    outs = []
    try:
        H_.call("ppo_tune_set", b"fc_splitk", Z)
        nb = H_.call("ppo_fc_fwd_ws_bytes", B, H)
        for tile in (1, 0):
            H_.call("ppo_tune_set", b"fc_splitk_tile", tile)
            ws = torch.full((nb // 4,), float("nan"), device=gpu)
            out = torch.full((B, H), float("nan"), device=gpu)
            H_.call("ppo_fc_fwd_ws", xd.data_ptr(), B, pk[2], bd.data_ptr(), H, out.data_ptr(), H, ws.data_ptr(), nb,
                    _s())
            torch.cuda.synchronize()
            outs.append(out)
    finally:
        H_.call("ppo_tune_set", b"fc_splitk", old[0])
        H_.call("ppo_tune_set", b"fc_splitk_tile", old[1])
    assert not torch.isnan(outs[0]).any()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("Z,cols", [(7, 100), (39, 802816), (96, 9000), (512, 512), (512, 1), (300, 4096), (1, 33)])
def test_colsum_vs_float64(gpu, Z, cols):
    """ppo_colsum (the deterministic split-K / block-partial reduce behind every
    weight gradient and the heads' partials) over the slab counts and widths the
    engine uses: within fp32 summation noise of float64 and the same bits twice."""
    H_ = _hip()
    g = torch.Generator().manual_seed(Z + cols)
    ld = cols + 3
    src = torch.randn(Z, ld, generator=g).cuda()
    outs = []
    for _ in range(2):
        out = torch.full((cols,), float("nan"), device=gpu)
        H_.call("ppo_colsum", src.data_ptr(), ld, Z, cols, out.data_ptr(), 0.5, 0, _s())
        outs.append(out)
    torch.cuda.synchronize()
    ref = 0.5 * src[:, :cols].double().sum(0)
    err = (outs[0].double() - ref).abs().max().item()
    assert err <= 1e-6 * Z * src.abs().max().item() + 1e-7
    assert torch.equal(outs[0], outs[1])


def _pack_mask3(a3):
    """conv3 output [B, 1568] (HWC: feature 32 p + c) -> the uint16 [B][49][2] mask words of
    ppo_conv3_fwd_mask (bit j of word (p, t): channel 16 t + j of pixel p > 0), as int32 [B, 98]"""
    bits = (a3 > 0).view(a3.shape[0], 98, 16).to(torch.int64)
    return (bits << torch.arange(16)).sum(-1).to(torch.int32)


@pytest.mark.parametrize("B", [300, 17, 4096, 3])
def test_conv3_fwd_mask_bits(gpu, B):
    """ppo_conv3_fwd_mask: the same output as ppo_conv3_fwd (bit-identical; B = 3 takes the
    image-resident kernel instead of the small-batch path, which is within fp32 tolerance)
    and the ReLU bits of exactly that output, lone output (6, 6) included"""
    H_ = _hip()
    w4, packed, pk = _packed(gpu, 64, 13)
    g = torch.Generator().manual_seed(B)
    a2 = torch.relu(torch.randn(B, 81 * 64, generator=g)).cuda()
    b3 = (torch.randn(32, generator=g) * 0.1).cuda()
    out = torch.full((B, 1568), float("nan"), device=gpu)
    ref = torch.full((B, 1568), float("nan"), device=gpu)
    m3 = torch.full((B * 49,), -1, dtype=torch.int32, device=gpu)
    H_.call("ppo_conv3_fwd_mask", a2.data_ptr(), B, pk[1], b3.data_ptr(), out.data_ptr(), m3.data_ptr(), _s())
    H_.call("ppo_conv3_fwd", a2.data_ptr(), B, pk[1], b3.data_ptr(), ref.data_ptr(), _s())
    torch.cuda.synchronize()
    if B > 4:
        assert torch.equal(out, ref)
    else:
        assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    got = m3.cpu().view(torch.int16).view(B, 98).to(torch.int32) & 0xFFFF
    assert torch.equal(got, _pack_mask3(out.cpu()))
    assert (out > 0).any() and (out == 0).any()


@pytest.mark.parametrize("B,H", [(300, 512), (77, 64), (200, 40)])
def test_fc_dgrad_bits_equals_act_mask(gpu, B, H):
    """ppo_fc_dgrad_bits (conv3's mask bits) == ppo_linear_dgrad_mask(act = a3), bit for bit"""
    H_ = _hip()
    w4, packed, pk = _packed(gpu, H, 5 + H)
    g = torch.Generator().manual_seed(B + 2)
    dh = torch.randn(B, H, generator=g).cuda()
    a3 = torch.relu(torch.randn(B, 1568, generator=g))
    m3 = _pack_mask3(a3).to(torch.int16).contiguous().cuda()   # the uint16 words [B][98] (bit patterns)
    a3d = a3.cuda()
    got = torch.full((B, 1568), float("nan"), device=gpu)
    ref = torch.full((B, 1568), float("nan"), device=gpu)
    H_.call("ppo_fc_dgrad_bits", dh.data_ptr(), B, H, pk[3], m3.data_ptr(), got.data_ptr(), _s())
    H_.call("ppo_linear_dgrad_mask", dh.data_ptr(), B, H, pk[3], 1568, a3d.data_ptr(), ref.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
