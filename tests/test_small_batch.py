"""Small-batch forward path (small.hip; SURVEY §8f f4, the batch-1 evaluation
act of T/run_evaluation.py:25-122): conv1 / conv2 / conv3 / fc / Linear at
B <= ppo_tune_get("small_b") against torch float64 (F.conv2d / linear), and
against the large-batch kernels with the small path switched off.  Tolerance:
max |err| <= 1e-5 * max |ref| (fp32 FMA sums of at most 1,568 terms)."""
import pytest
import torch
import torch.nn.functional as F

from test_gpu_parity import _hip, _packed, _s

pytestmark = pytest.mark.gpu


def _close(got, ref, tol=1e-5):
    err = (got.cpu().double() - ref).abs().max().item()
    assert err <= tol * max(ref.abs().max().item(), 1e-30), err


def _both(fn):
    """fn() with the small path on (default) and off (small_b = 0)."""
    Hh = _hip()
    old = Hh.call("ppo_tune_get", b"small_b")
    assert old >= 1
    try:
        on = fn()
        Hh.call("ppo_tune_set", b"small_b", 0)
        off = fn()
    finally:
        Hh.call("ppo_tune_set", b"small_b", old)
    torch.cuda.synchronize()
    return on, off


@pytest.mark.parametrize("B", [1, 3])
@pytest.mark.parametrize("u8", [True, False])
def test_small_conv_trunk_vs_torch(gpu, B, u8):
    Hh = _hip()
    H = 256
    w, packed, pk = _packed(gpu, H, 91)
    g = torch.Generator().manual_seed(92)
    rows = 7
    obs = (torch.randint(0, 256, (rows, 4, 84, 84), dtype=torch.uint8, generator=g) if u8
           else torch.rand(rows, 4, 84, 84, generator=g))
    idx = torch.randperm(rows, generator=g)[:B].contiguous()
    w1, b1 = torch.randn(32, 4, 8, 8, generator=g) * 0.05, torch.randn(32, generator=g) * 0.1
    b2, b3, b4 = (torch.randn(n, generator=g) * 0.1 for n in (64, 32, H))
    d = {k: v.cuda() for k, v in dict(obs=obs, idx=idx, w1=w1, b1=b1, b2=b2, b3=b3, b4=b4).items()}

    def run():
        a1 = torch.full((B, 20, 20, 32), float("nan"), device=gpu)
        a2 = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
        a3 = torch.full((B, 7, 7, 32), float("nan"), device=gpu)
        h = torch.full((B, H), float("nan"), device=gpu)
        Hh.call("ppo_conv1_fwd", d["obs"].data_ptr(), int(u8), d["idx"].data_ptr(), 0, 4, B, d["w1"].data_ptr(),
                d["b1"].data_ptr(), a1.data_ptr(), _s())
        Hh.call("ppo_conv2_fwd", a1.data_ptr(), B, pk[0], d["b2"].data_ptr(), a2.data_ptr(), _s())
        Hh.call("ppo_conv3_fwd", a2.data_ptr(), B, pk[1], d["b3"].data_ptr(), a3.data_ptr(), _s())
        Hh.call("ppo_fc_fwd", a3.data_ptr(), B, pk[2], d["b4"].data_ptr(), H, h.data_ptr(), H, _s())
        return a1, a2, a3, h

    on, off = _both(run)
    x = obs[idx].double() / (255.0 if u8 else 1.0)
    r1 = torch.relu(F.conv2d(x, w1.double(), b1.double(), stride=4))
    r2 = torch.relu(F.conv2d(r1, w["w2"].double(), b2.double(), stride=2))
    r3 = torch.relu(F.conv2d(r2, w["w3"].double(), b3.double()))
    r4 = torch.relu(F.linear(r3.reshape(B, -1), w["w4"].double(), b4.double()))   # torch flatten: (c, y, x)
    # each layer against torch on the previous layer's HIP output (no error build-up)
    refs_on = [r1.permute(0, 2, 3, 1),
               torch.relu(F.conv2d(on[0].cpu().double().permute(0, 3, 1, 2), w["w2"].double(), b2.double(),
                                   stride=2)).permute(0, 2, 3, 1),
               torch.relu(F.conv2d(on[1].cpu().double().permute(0, 3, 1, 2), w["w3"].double(),
                                   b3.double())).permute(0, 2, 3, 1),
               torch.relu(F.linear(on[2].cpu().double().permute(0, 3, 1, 2).reshape(B, -1), w["w4"].double(),
                                   b4.double()))]
    for got, ref in zip(on, refs_on):
        assert not torch.isnan(got).any()
        _close(got, ref)
    _close(on[3], r4, 1e-4)
    for a, b in zip(on, off):   # the small path and the MFMA kernels agree
        _close(a, b.cpu().double(), 1e-4)


@pytest.mark.parametrize("act", [0, 1, 2])
def test_small_linear_ex_vs_torch(gpu, act):
    """ppo_linear_fwd_ex at M = 2 with a row gather, row strides and each
    activation (the GRU input projection and the MLP layers of the act path)."""
    Hh = _hip()
    g = torch.Generator().manual_seed(93)
    M, K, N, lda, ldo = 2, 268, 768, 272, 770
    x = torch.randn(5, lda, generator=g)
    idx = torch.tensor([3, 1], dtype=torch.int64)
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g) * 0.1
    xd, idxd, wd, bd = x.cuda(), idx.cuda(), w.cuda(), b.cuda()

    def run():
        out = torch.full((M, ldo), float("nan"), device=gpu)
        Hh.call("ppo_linear_fwd_ex", xd.data_ptr(), idxd.data_ptr(), M, K, lda, wd.data_ptr(), bd.data_ptr(), N,
                out.data_ptr(), ldo, act, _s())
        return out

    on, off = _both(run)
    ref = F.linear(x[idx, :K].double(), w.double(), b.double())
    ref = torch.relu(ref) if act == 1 else torch.tanh(ref) if act == 2 else ref
    _close(on[:, :N], ref)
    _close(off[:, :N], ref)
    assert torch.isnan(on[:, N:]).all()   # untouched beyond N in each row


def test_small_path_graph_and_eager_act_agree(gpu):
    """The batch-1 evaluation act (GraphedActor over the small path) equals the
    eager act bit for bit and, with the small path off, the MFMA path within
    the fp32 tolerance."""
    from a2c_ppo_acktr.evaluation import GraphedActor
    from a2c_ppo_acktr.model import CNNBase, Policy
    from a2c_ppo_acktr.synthetic import Discrete
    Hh = _hip()
    torch.manual_seed(5)
    pol = Policy((4, 84, 84), Discrete(8), base=CNNBase, base_kwargs={"recurrent": True, "hidden_size": 256},
                 vector_obs_len=14)
    pol.to(gpu)
    obs = torch.rand(1, 4, 84, 84, device=gpu)
    vec, h, m = torch.rand(1, 14, device=gpu), torch.rand(1, 256, device=gpu), torch.ones(1, 1, device=gpu)
    ga = GraphedActor(pol)
    with torch.no_grad():
        e = pol.act(obs, vec, h, m, deterministic=True)
        r = ga.act(obs, vec, h, m)
        torch.cuda.synchronize()
        for a, b in zip(e, r):
            assert torch.equal(a, b)
        old = Hh.call("ppo_tune_get", b"small_b")
        Hh.call("ppo_tune_set", b"small_b", 0)
        try:
            big = pol.act(obs, vec, h, m, deterministic=True)
            torch.cuda.synchronize()
        finally:
            Hh.call("ppo_tune_set", b"small_b", old)
    assert torch.equal(e[1], big[1])
    for a, b in ((e[0], big[0]), (e[3], big[3])):
        assert (a - b).abs().max().item() <= 1e-4 * max(b.abs().max().item(), 1.0)
