"""conv1 -> conv2 with conv1's output pre-split (csrc/a1split.hip).  The split
path must be bit-identical to the fp32-a1 path it replaces (conv1's sums are
the same MFMA products with swapped operands, the split is the consumers' own
split8 arithmetic, and the consumers' products and summation orders are
unchanged), which itself is held to torch float64 in test_gpu_parity.py /
test_full_size.py.  Reference: CNNBase conv1 -> conv2, T/a2c_ppo_acktr/model.py:177-180.

* conv1: a1s planes == the exact bf16 split (RNE residuals) of ppo_conv1_fwd_mask's
  fp32 a1, in the documented unit order; the mask bits are equal;
* conv2 forward from a1s (LDS-DMA staged) == ppo_conv2_fwd_mask from a1, output
  and mask bits;
* conv2 weight gradient from a1s == ppo_conv2_wgrad from a1 (slabs);
* a whole training minibatch and a rollout act through the engine: gradients,
  losses and act outputs bit-identical with the tune knob on and off."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    from a2c_ppo_acktr import _hip
    return _hip


def _s():
    return torch.cuda.current_stream().cuda_stream


def _rho(y, x):
    return 100 * (2 * (y & 1) + (x & 1)) + 10 * (y >> 1) + (x >> 1)


def _split_planes(a1):
    """exact three-way bf16 split (RNE at each residual) of fp32 [B][20][20][32]
    -> int16 bit patterns [3][B][20][20][32]"""
    h = a1.to(torch.bfloat16)
    r = a1 - h.float()
    m = r.to(torch.bfloat16)
    r2 = r - m.float()
    l_ = r2.to(torch.bfloat16)
    return torch.stack([t.view(torch.int16) for t in (h, m, l_)])


def _a1s_expected(a1):
    """[B][4800 units][8] int16 in the documented order: unit (p, c, rho(y, x))"""
    B = a1.shape[0]
    pl = _split_planes(a1).cpu()
    out = torch.zeros(B, 3, 4, 400, 8, dtype=torch.int16)
    ys, xs = np.meshgrid(np.arange(20), np.arange(20), indexing="ij")
    rho = torch.from_numpy(_rho(ys, xs).reshape(-1))
    v = pl.reshape(3, B, 400, 4, 8).permute(1, 0, 3, 2, 4)   # [B][p][c][pixel y*20+x][8]
    out[:, :, :, rho, :] = v
    return out.reshape(B, 4800, 8)


@pytest.fixture
def split_on():
    Hh = _hip()
    old = Hh.call("ppo_tune_get", b"a1split")
    yield Hh
    Hh.call("ppo_tune_set", b"a1split", old)


def _conv1_inputs(gpu, B, seed):
    g = torch.Generator().manual_seed(seed)
    rows = 3 * B + 7
    obs = torch.randint(0, 256, (rows, 4, 84, 84), dtype=torch.uint8, generator=g).to(gpu)
    idx = torch.randperm(rows, generator=g)[:B].to(gpu)
    w1 = (torch.randn(32, 256, generator=g) * 0.05).to(gpu)
    b1 = (torch.randn(32, generator=g) * 0.1).to(gpu)
    return obs, idx, w1, b1


@pytest.mark.parametrize("B", [300, 5, 257])
def test_conv1_split_planes_and_mask(gpu, split_on, B):
    Hh = split_on
    obs, idx, w1, b1 = _conv1_inputs(gpu, B, 3)
    a1 = torch.empty(B, 20, 20, 32, device=gpu)
    m_ref = torch.zeros(B * 400, dtype=torch.int32, device=gpu)
    Hh.call("ppo_conv1_fwd_mask", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
            a1.data_ptr(), m_ref.data_ptr(), _s())
    a1s = torch.full((Hh.call("ppo_a1s_bytes", B) // 2,), -1, dtype=torch.int16, device=gpu)
    m = torch.zeros(B * 400, dtype=torch.int32, device=gpu)
    Hh.call("ppo_conv1_fwd_split", obs.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(), b1.data_ptr(),
            a1s.data_ptr(), m.data_ptr(), _s())
    torch.cuda.synchronize()
    exp = _a1s_expected(a1)
    got = a1s.cpu().reshape(B, 4800, 8)
    assert torch.equal(got, exp), int((got != exp).sum())
    assert torch.equal(m, m_ref)
    # the act form (no mask) writes the same planes
    a1s2 = torch.full_like(a1s, -1)
    Hh.call("ppo_conv1_fwd_split", obs.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(), b1.data_ptr(),
            a1s2.data_ptr(), None, _s())
    torch.cuda.synchronize()
    assert torch.equal(a1s2, a1s)


def _packed(gpu, seed):
    Hh = _hip()
    g = torch.Generator().manual_seed(seed)
    w2 = (torch.randn(64, 32, 4, 4, generator=g) * 0.05).to(gpu)
    w3 = (torch.randn(32, 64, 3, 3, generator=g) * 0.05).to(gpu)
    w4 = (torch.randn(64, 1568, generator=g) * 0.02).to(gpu)
    packed = torch.zeros(Hh.call("ppo_packed_weights_size", 64), device=gpu)
    offs = torch.zeros(6, dtype=torch.int64)
    Hh.call("ppo_packed_offsets", 64, offs.data_ptr())
    Hh.call("ppo_pack_weights", w2.data_ptr(), w3.data_ptr(), w4.data_ptr(), 64, packed.data_ptr(), _s())
    return packed, [packed.data_ptr() + 4 * int(o) for o in offs]


@pytest.mark.parametrize("products", [6, 9])
@pytest.mark.parametrize("B", [300, 3, 513])
def test_conv2_fwd_split_equals_fp32_path(gpu, split_on, B, products):
    Hh = split_on
    old_np = Hh.call("ppo_tune_get", b"products")
    Hh.call("ppo_tune_set", b"products", products)
    try:
        obs, idx, w1, b1 = _conv1_inputs(gpu, B, 5)
        packed, pk = _packed(gpu, 6)
        b2 = (torch.randn(64, generator=torch.Generator().manual_seed(7)) * 0.1).to(gpu)
        a1 = torch.empty(B, 20, 20, 32, device=gpu)
        m1 = torch.empty(B * 400, dtype=torch.int32, device=gpu)   # the image-resident kernel at any B
        Hh.call("ppo_conv1_fwd_mask", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
                a1.data_ptr(), m1.data_ptr(), _s())
        a1s = torch.empty(Hh.call("ppo_a1s_bytes", B) // 2, dtype=torch.int16, device=gpu)
        Hh.call("ppo_conv1_fwd_split", obs.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(), b1.data_ptr(),
                a1s.data_ptr(), None, _s())
        ref = torch.full((B, 81, 64), float("nan"), device=gpu)
        mref = torch.zeros(B * 81, dtype=torch.int64, device=gpu)
        out = torch.full_like(ref, float("nan"))
        mb = torch.zeros_like(mref)
        Hh.call("ppo_conv2_fwd_mask", a1.data_ptr(), B, pk[0], b2.data_ptr(), ref.data_ptr(), mref.data_ptr(), _s())
        Hh.call("ppo_conv2_fwd_split", a1s.data_ptr(), B, pk[0], b2.data_ptr(), out.data_ptr(), mb.data_ptr(), _s())
        out2 = torch.full_like(ref, float("nan"))
        Hh.call("ppo_conv2_fwd_split", a1s.data_ptr(), B, pk[0], b2.data_ptr(), out2.data_ptr(), None, _s())
        torch.cuda.synchronize()
        assert torch.equal(out, ref), float((out - ref).abs().max())
        assert torch.equal(out2, ref)
        assert torch.equal(mb, mref)
    finally:
        Hh.call("ppo_tune_set", b"products", old_np)


@pytest.mark.parametrize("B", [300, 1000])
def test_conv2_wgrad_split_equals_fp32_path(gpu, split_on, B):
    Hh = split_on
    obs, idx, w1, b1 = _conv1_inputs(gpu, B, 9)
    a1 = torch.empty(B, 20, 20, 32, device=gpu)
    Hh.call("ppo_conv1_fwd", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
            a1.data_ptr(), _s())
    a1s = torch.empty(Hh.call("ppo_a1s_bytes", B) // 2, dtype=torch.int16, device=gpu)
    Hh.call("ppo_conv1_fwd_split", obs.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(), b1.data_ptr(),
            a1s.data_ptr(), None, _s())
    dz2 = torch.randn(B, 9, 9, 64, generator=torch.Generator().manual_seed(10)).to(gpu)
    Z = min(B, 256)
    slabs = []
    for name, x in (("ppo_conv2_wgrad", a1), ("ppo_conv2_wgrad_split", a1s)):
        slab = torch.full((Z * 64 * 512,), float("nan"), device=gpu)
        slab_b = torch.full((Z * 64,), float("nan"), device=gpu)
        Hh.call(name, dz2.data_ptr(), x.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), _s())
        slabs.append((slab, slab_b))
    torch.cuda.synchronize()
    assert torch.equal(slabs[0][0], slabs[1][0])
    assert torch.equal(slabs[0][1], slabs[1][1])


class _GradCapture(object):
    def _step_flat(self, eng):
        self.grad = eng.grad.clone()


def test_engine_minibatch_and_act_bit_identical(gpu, split_on):
    """one training minibatch (gradient + losses) and one rollout act through
    CNNEngine with the split hand-off on and off"""
    Hh = split_on
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    H, T, N, A = 512, 8, 512, 8
    torch.manual_seed(4)
    pol = M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    pol.to(gpu)
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(A), 1, obs_dtype=torch.uint8, device=gpu)
    g = torch.Generator().manual_seed(5)
    st.obs.copy_(torch.randint(0, 256, st.obs.shape, dtype=torch.uint8, generator=g).to(gpu))
    st.actions.copy_(torch.randint(0, A, st.actions.shape, generator=g).to(gpu))
    st.action_log_probs.copy_((torch.log(torch.rand(st.action_log_probs.shape, generator=g)) * 0.3 - 2.0).to(gpu))
    st.value_preds.copy_(torch.randn(st.value_preds.shape, generator=g).to(gpu) * 0.1)
    st.returns.copy_(torch.randn(st.returns.shape, generator=g).to(gpu))
    adv = torch.randn(T, N, generator=torch.Generator().manual_seed(6)).to(gpu)
    idx = torch.randperm(T * N, generator=torch.Generator().manual_seed(7))[:2048].to(gpu)
    hp = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.01, "use_clipped_value_loss": True}
    eng = pol.hip_engine()
    res = {}
    for on in (0, 1):
        Hh.call("ppo_tune_set", b"a1split", on)
        loss = torch.zeros(4, dtype=torch.float64, device=gpu)
        cap = _GradCapture()
        eng.train_minibatch(st, adv, idx, hp, loss, cap)
        noise = torch.empty(N, A).exponential_(1, generator=torch.Generator().manual_seed(8))
        v, a, lp, _ = eng.act(st.obs[0], noise=noise)
        torch.cuda.synchronize()
        res[on] = (cap.grad.clone(), loss.clone(), v.clone(), a.clone(), lp.clone())
    assert "a1s" in eng.ws["train"].bufs and "a1s" in eng.ws[eng.act_ws].bufs
    for x, y in zip(res[0], res[1]):
        assert torch.equal(x, y)
