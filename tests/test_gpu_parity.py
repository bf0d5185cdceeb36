"""GPU parity: every HIP kernel through the C ABI against the oracle (and the
reference's golden vectors).  Tolerances are stated per test; integer/index work
and GAE are bit-exact."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import ppo_oracle as O

pytestmark = pytest.mark.gpu


def _hip():
    from a2c_ppo_acktr import _hip
    return _hip


def _s():
    return torch.cuda.current_stream().cuda_stream


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


# ---------------------------------------------------------------- GAE (K3/K4)
@pytest.mark.parametrize("gi", [0, 1])
@pytest.mark.parametrize("use_gae", [True, False])
@pytest.mark.parametrize("ptl", [True, False])
def test_gae_golden_bit_exact(gpu, gi, use_gae, ptl):
    H = _hip()
    d = golden("gae.npz")
    T, N = d["rewards"].shape[:2]
    r, v, m, bm = (_dev(d[k][..., 0]) for k in ("rewards", "value_preds", "masks", "bad_masks"))
    nv = _dev(d["next_value"][:, 0])
    ret = torch.full((T + 1, N), -7.0, device=gpu)
    H.call("ppo_compute_returns", r.data_ptr(), v.data_ptr(), m.data_ptr(), bm.data_ptr(), nv.data_ptr(),
           ret.data_ptr(), None, None, T, N, float(d["gammas"][gi]), float(d["lambdas"][gi]), int(use_gae),
           int(ptl), _s())
    k = f"g{gi}_gae{int(use_gae)}_ptl{int(ptl)}"
    assert np.array_equal(ret.cpu().numpy(), d[k + "_returns"][..., 0])
    assert np.array_equal(v.cpu().numpy(), d[k + "_value_preds"][..., 0])


@pytest.mark.parametrize("T,N", [(128, 4096), (5, 1), (1, 300), (77, 1031)])
def test_gae_fused_adv_vs_oracle(gpu, T, N):
    """bit-exact returns at the c3 shape and ragged shapes; fused advantage
    statistics within 1e-6 (the reference reduces in float, we in double)."""
    H = _hip()
    rng = np.random.default_rng(T * 7 + N)
    r = rng.random((T, N), np.float32)
    v = (3 * rng.standard_normal((T + 1, N))).astype(np.float32)
    m = (rng.random((T + 1, N)) > 0.01).astype(np.float32)
    bm = np.ones((T + 1, N), np.float32)
    nv = rng.standard_normal(N).astype(np.float32)
    rd, vd, md, bmd, nvd = _dev(r), _dev(v), _dev(m), _dev(bm), _dev(nv)
    ret = torch.zeros(T + 1, N, device=gpu)
    adv = torch.zeros(T, N, device=gpu)
    nparts = H.call("ppo_gae_partials_count", N)
    parts = torch.zeros(3 * nparts, dtype=torch.float64, device=gpu)
    stats = torch.zeros(3, dtype=torch.float64, device=gpu)
    H.call("ppo_compute_returns", rd.data_ptr(), vd.data_ptr(), md.data_ptr(), bmd.data_ptr(), nvd.data_ptr(),
           ret.data_ptr(), adv.data_ptr(), parts.data_ptr(), T, N, 0.99, 0.95, 1, 0, _s())
    H.call("ppo_adv_finalize", parts.data_ptr(), nparts, float(T * N), stats.data_ptr(), _s())
    H.call("ppo_adv_normalize", adv.data_ptr(), T * N, stats.data_ptr(), _s())
    eret, ev = O.compute_returns(r, v, m, bm, nv, True, 0.99, 0.95, False)
    assert np.array_equal(ret.cpu().numpy()[:T], eret[:T])
    assert np.array_equal(vd.cpu().numpy(), ev)
    if T * N > 1:
        np.testing.assert_allclose(adv.cpu().numpy(), O.normalize_advantages(eret, ev), rtol=1e-6, atol=1e-6)


def test_advnorm_golden(gpu):
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("advnorm.npz")
    for c in range(3):
        ret, val = d[f"c{c}_returns"], d[f"c{c}_value_preds"]
        T, N = ret.shape[0] - 1, ret.shape[1]
        st = RolloutStorage(T, N, (1,), [0], Discrete(2), 1, device=gpu)
        st.returns.copy_(_dev(ret))
        st.value_preds.copy_(_dev(val))
        adv = st.normalized_advantages()
        np.testing.assert_allclose(adv.cpu().numpy(), d[f"c{c}_advantages"][..., 0], rtol=1e-6, atol=1e-6)


# ------------------------------------------------------------- storage (K1/K2/K5/K6)
def test_sampler_golden_bit_exact(gpu):
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("sampler.npz")
    for c in range(4):
        seed, T, N, M = (int(x) for x in d[f"c{c}_meta"])
        st = RolloutStorage(T, N, (1,), [0], Discrete(2), 1, device=gpu)
        st.value_preds[:-1].copy_(torch.arange(T * N, dtype=torch.float32, device=gpu).view(T, N, 1))
        adv = torch.zeros(T, N, 1, device=gpu)
        torch.manual_seed(seed)
        ff = np.stack([b[4].view(-1).long().cpu().numpy() for b in st.feed_forward_generator(adv, M)])
        assert np.array_equal(ff, d[f"c{c}_ff"])
        if f"c{c}_rec" in d:
            torch.manual_seed(seed)
            rec = np.stack([b[4].view(-1).long().cpu().numpy() for b in st.recurrent_generator(adv, M)])
            assert np.array_equal(rec, d[f"c{c}_rec"])


def test_generator_gathers_every_field(gpu):
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    T, N, M = 6, 5, 3
    st = RolloutStorage(T, N, (4, 84, 84), [3], Discrete(8), 2, obs_dtype=torch.uint8, device=gpu)
    g = torch.Generator().manual_seed(0)
    st.obs.copy_(torch.randint(0, 256, st.obs.shape, dtype=torch.uint8, generator=g).to(gpu))
    for t in (st.vector_obs, st.recurrent_hidden_states, st.value_preds, st.returns, st.masks, st.action_log_probs):
        t.copy_(torch.randn(t.shape, generator=g).to(gpu))
    st.actions.copy_(torch.randint(0, 8, st.actions.shape, generator=g).to(gpu))
    adv = torch.randn(T, N, 1, generator=g).to(gpu)
    torch.manual_seed(3)
    batches = list(st.feed_forward_generator(adv, M))
    torch.manual_seed(3)
    perm = torch.randperm(T * N)
    mb = T * N // M
    for i, b in enumerate(batches):
        idx = perm[i * mb:(i + 1) * mb].to(gpu)
        exp = [st.obs[:-1].reshape(T * N, 4, 84, 84)[idx], st.vector_obs[:-1].reshape(T * N, 3)[idx],
               st.recurrent_hidden_states[:-1].reshape(T * N, 2)[idx], st.actions.reshape(T * N, 1)[idx],
               st.value_preds[:-1].reshape(-1, 1)[idx], st.returns[:-1].reshape(-1, 1)[idx],
               st.masks[:-1].reshape(-1, 1)[idx], st.action_log_probs.reshape(-1, 1)[idx], adv.reshape(-1, 1)[idx]]
        for got, e in zip(b, exp):
            assert torch.equal(got, e)
    # recurrent generator: env columns, hxs from t=0
    st2 = RolloutStorage(T, 6, (4, 84, 84), [3], Discrete(8), 2, obs_dtype=torch.uint8, device=gpu)
    st2.obs.copy_(torch.randint(0, 256, st2.obs.shape, dtype=torch.uint8, generator=g).to(gpu))
    st2.recurrent_hidden_states.copy_(torch.randn(st2.recurrent_hidden_states.shape, generator=g).to(gpu))
    adv2 = torch.randn(T, 6, 1, generator=g).to(gpu)
    torch.manual_seed(4)
    batches = list(st2.recurrent_generator(adv2, 3))
    torch.manual_seed(4)
    perm = torch.randperm(6)
    for i, b in enumerate(batches):
        envs = perm[i * 2:(i + 1) * 2].to(gpu)
        assert torch.equal(b[0], st2.obs[:-1][:, envs].reshape(T * 2, 4, 84, 84))
        assert torch.equal(b[2], st2.recurrent_hidden_states[0][envs])
        assert torch.equal(b[8], adv2[:, envs].reshape(T * 2, 1))
    with pytest.raises(IndexError):
        list(RolloutStorage(2, 7, (1,), [0], Discrete(2), 1, device=gpu).recurrent_generator(
            torch.zeros(2, 7, 1, device=gpu), 3))


def test_insert_and_after_update(gpu):
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    T, N = 3, 5
    st = RolloutStorage(T, N, (4, 84, 84), [2], Discrete(8), 1, device=gpu)
    ref = {k: getattr(st, k).clone() for k in ("obs", "vector_obs", "recurrent_hidden_states", "actions",
                                               "action_log_probs", "value_preds", "rewards", "masks", "bad_masks")}
    g = torch.Generator().manual_seed(1)
    for step in range(T):
        o = torch.rand(N, 4, 84, 84, generator=g)
        vo = torch.rand(N, 2, generator=g)
        h = torch.rand(N, 1, generator=g)
        a = torch.randint(0, 8, (N, 1), generator=g)
        lp, v, r = torch.rand(N, 1, generator=g), torch.rand(N, 1, generator=g), torch.rand(N, 1, generator=g)
        mk = (torch.rand(N, 1, generator=g) > 0.5).float()
        bmk = (torch.rand(N, 1, generator=g) > 0.5).float()
        # host tensors on purpose (run.py passes CPU masks/rewards)
        st.insert(o, vo.cuda(), h.cuda(), a.cuda(), lp.cuda(), v.cuda(), r, mk, bmk)
        ref["obs"][step + 1] = o.cuda(); ref["vector_obs"][step + 1] = vo.cuda()
        ref["recurrent_hidden_states"][step + 1] = h.cuda(); ref["actions"][step] = a.cuda()
        ref["action_log_probs"][step] = lp.cuda(); ref["value_preds"][step] = v.cuda()
        ref["rewards"][step] = r.cuda(); ref["masks"][step + 1] = mk.cuda(); ref["bad_masks"][step + 1] = bmk.cuda()
    assert st.step == 0
    for k, t in ref.items():
        assert torch.equal(getattr(st, k), t), k
    st.after_update()
    for k in ("obs", "vector_obs", "recurrent_hidden_states", "masks", "bad_masks"):
        assert torch.equal(getattr(st, k)[0], ref[k][-1]), k


def _synth_ref(seed, step, N, nbytes, p_done):
    """numpy restatement of synth_env_kernel (storage.hip)"""
    M64 = (1 << 64) - 1

    def mix(z):
        z = (z + 0x9E3779B97F4A7C15) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    obs = np.zeros((N, nbytes), np.uint8)
    rew = np.zeros(N, np.float32)
    msk = np.zeros(N, np.float32)
    for n in range(N):
        key = seed ^ mix((step * 0x100000001B3 + n * 0x9E3779B1) & M64)
        words = []
        for c in range(nbytes // 8):
            words.append(mix((key + c) & M64))
        obs[n] = np.array(words, dtype=np.uint64).view(np.uint8)
        k = mix(seed ^ mix((step * 0x100000001B3 + n * 0x9E3779B1 + 0x5EED) & M64))
        u = (np.float32((k >> 40) & 0xFFFFFF) + np.float32(1)) * np.float32(1 / 16777216)
        rew[n] = u - np.float32(1 / 16777216)
        k2 = mix(k ^ 0xD0D0D0D0)
        u2 = (np.float32((k2 >> 40) & 0xFFFFFF) + np.float32(1)) * np.float32(1 / 16777216)
        msk[n] = 0.0 if u2 < np.float32(p_done) else 1.0
    return obs, rew, msk


def test_synthetic_env_reproducible(gpu):
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    N = 3
    env = SyntheticVecEnv(N, seed=99, p_done=0.5, device=gpu)
    slot = torch.zeros(N, 4, 84, 84, dtype=torch.uint8, device=gpu)
    env.counter = 5
    r, m, bm = env.step_into(slot)
    obs, rew, msk = _synth_ref(99, 5, N, 4 * 84 * 84, 0.5)
    assert np.array_equal(slot.cpu().numpy().reshape(N, -1), obs)
    assert np.array_equal(r.cpu().numpy()[:, 0], rew)
    assert np.array_equal(m.cpu().numpy()[:, 0], msk)
    assert torch.all(bm == 1)


# ------------------------------------------------------------- trunk (K7-K10, K16)
def _cnn_params(H, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    shapes = O.cnn_param_shapes(H)
    flat = torch.cat([torch.randn(int(np.prod(s)), generator=g) * (scale / np.sqrt(np.prod(s[1:]) if len(s) > 1
                                                                                    else 1.0))
                      for _, s in shapes])
    return flat.numpy().astype(np.float32), shapes


@pytest.mark.parametrize("B,H", [(8, 64), (37, 512)])
def test_trunk_forward_vs_torch_fp32(gpu, B, H):
    """conv1..fc forward through the ABI vs torch fp32 (same op, plain PyTorch);
    tolerance 2e-5 relative to the activation scale (fp32, different sum order)."""
    Hh = _hip()
    flat, shapes = _cnn_params(H, seed=B)
    p = {n: torch.from_numpy(v.astype(np.float32)) for n, v in O.unflatten(flat, shapes, np.float32).items()}
    g = torch.Generator().manual_seed(B)
    obs_u8 = torch.randint(0, 256, (B + 3, 4, 84, 84), dtype=torch.uint8, generator=g)
    idx = torch.randperm(B + 3, generator=g)[:B]
    x = obs_u8[idx].float() / 255.0
    a1 = F.relu(F.conv2d(x, p["base.main.0.weight"], p["base.main.0.bias"], stride=4))
    a2 = F.relu(F.conv2d(a1, p["base.main.2.weight"], p["base.main.2.bias"], stride=2))
    a3 = F.relu(F.conv2d(a2, p["base.main.4.weight"], p["base.main.4.bias"], stride=1))
    hh = F.relu(a3.reshape(B, -1) @ p["base.main.7.weight"].t() + p["base.main.7.bias"])
    d = {k: v.cuda() for k, v in p.items()}
    packed = torch.empty(Hh.call("ppo_packed_weights_size", H), device=gpu)
    offs = torch.zeros(6, dtype=torch.int64)
    Hh.call("ppo_packed_offsets", H, offs.data_ptr())
    pk = [packed.data_ptr() + 4 * int(o) for o in offs]
    Hh.call("ppo_pack_weights", d["base.main.2.weight"].data_ptr(), d["base.main.4.weight"].data_ptr(),
            d["base.main.7.weight"].data_ptr(), H, packed.data_ptr(), _s())
    obs_d, idx_d = obs_u8.cuda(), idx.cuda()
    o1 = torch.empty(B, 20, 20, 32, device=gpu)
    o2 = torch.empty(B, 9, 9, 64, device=gpu)
    o3 = torch.empty(B, 7, 7, 32, device=gpu)
    o4 = torch.empty(B, H, device=gpu)
    Hh.call("ppo_conv1_fwd", obs_d.data_ptr(), 1, idx_d.data_ptr(), 0, 4, B, d["base.main.0.weight"].data_ptr(),
            d["base.main.0.bias"].data_ptr(), o1.data_ptr(), _s())
    Hh.call("ppo_conv2_fwd", o1.data_ptr(), B, pk[0], d["base.main.2.bias"].data_ptr(), o2.data_ptr(), _s())
    Hh.call("ppo_conv3_fwd", o2.data_ptr(), B, pk[1], d["base.main.4.bias"].data_ptr(), o3.data_ptr(), _s())
    Hh.call("ppo_fc_fwd", o3.data_ptr(), B, pk[2], d["base.main.7.bias"].data_ptr(), H, o4.data_ptr(), H, _s())
    for got, ref in ((o1, a1.permute(0, 2, 3, 1)), (o2, a2.permute(0, 2, 3, 1)), (o3, a3.permute(0, 2, 3, 1)),
                     (o4, hh)):
        ref = ref.contiguous()
        err = (got.cpu() - ref).abs().max().item()
        assert err <= 2e-5 * max(1.0, ref.abs().max().item()), err
    # f32 observation path (reference convention: pre-normalised floats)
    xf = (obs_u8.float() / 255.0).cuda()
    o1f = torch.empty_like(o1)
    Hh.call("ppo_conv1_fwd", xf.data_ptr(), 0, idx_d.data_ptr(), 0, 4, B, d["base.main.0.weight"].data_ptr(),
            d["base.main.0.bias"].data_ptr(), o1f.data_ptr(), _s())
    # u8 path folds the 1/255 into the accumulator: within fp32 rounding of the f32 path
    assert (o1f - o1).abs().max().item() <= 2e-6 * max(1.0, o1.abs().max().item())


@pytest.mark.parametrize("B,H", [(6, 64), (33, 512)])
def test_loss_and_backward_vs_oracle(gpu, B, H):
    """Fused heads/loss + every dgrad/wgrad kernel (through the engine) vs the
    oracle's float64 analytic backward: max |err| <= 1e-5 * max|grad| per tensor."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo.ppo import FlatAdam
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    torch.manual_seed(B)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    with torch.no_grad():   # widen the heads so every loss branch carries weight
        pol.dist.linear.weight.mul_(50.0)
        pol.base.critic_linear.weight.mul_(3.0)
    init = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy().astype(np.float64)
    pol.to(gpu)
    eng = pol.hip_engine()
    T, N = 3, B
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), 1, obs_dtype=torch.uint8, device=gpu)
    g = torch.Generator().manual_seed(B + 1)
    st.obs.copy_(torch.randint(0, 256, st.obs.shape, dtype=torch.uint8, generator=g).to(gpu))
    st.actions.copy_(torch.randint(0, 8, st.actions.shape, generator=g).to(gpu))
    st.action_log_probs.copy_((torch.log(torch.rand(st.action_log_probs.shape, generator=g)) * 0.3 - 2.0).to(gpu))
    st.value_preds.copy_(torch.randn(st.value_preds.shape, generator=g).to(gpu) * 0.1)
    st.returns.copy_(torch.randn(st.returns.shape, generator=g).to(gpu))
    adv = torch.randn(T, N, generator=g).to(gpu)
    idx = torch.randperm(T * N, generator=g)[: (T * N) // 2].to(gpu)
    hp = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.01, "use_clipped_value_loss": True}
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)   # 3 losses + bad-action count
    opt = FlatAdam(pol.parameters(), lr=0.0, eps=1e-5, max_grad_norm=None)  # lr 0: grads only
    eng.train_minibatch(st, adv, idx, hp, loss, opt)
    torch.cuda.synchronize()
    shapes = O.cnn_param_shapes(H)
    p = O.unflatten(init, shapes)
    ii = idx.cpu().numpy()
    obs = st.obs[:-1].reshape(T * N, 4, 84, 84).cpu().numpy()[ii]
    value, logits, cache = O.cnn_forward(p, O.decode_obs(obs))
    f = lambda t: t.reshape(-1).cpu().numpy()[ii]  # noqa: E731
    lg = O.loss_head_grads(value, logits, f(st.actions), f(st.action_log_probs), f(adv),
                           st.value_preds[:-1].reshape(-1).cpu().numpy()[ii],
                           st.returns[:-1].reshape(-1).cpu().numpy()[ii], 0.1, 0.5, 0.01)
    grads = O.cnn_backward(p, cache, lg["g_value"], lg["g_logits"])
    got = O.unflatten(eng.grad.cpu().numpy(), shapes)
    for name, _ in shapes:
        ref = grads[name]
        err = np.abs(got[name] - ref).max()
        assert err <= 1e-5 * max(np.abs(ref).max(), 1e-3), (name, err, np.abs(ref).max())
    np.testing.assert_allclose(loss.cpu().numpy()[:3], [lg["value_loss"], lg["action_loss"], lg["entropy"]],
                               rtol=2e-5, atol=1e-6)


# ------------------------------------------------------------------ heads (K13/K14)
def test_categorical_golden(gpu):
    Hh = _hip()
    d = golden("categorical.npz")
    feats = d["features"]
    N, Hd = feats.shape
    A = d["weight"].shape[0]
    Hp = 64   # kernel needs H % 64 == 0: zero-pad the feature dimension
    f = np.zeros((N, Hp), np.float32); f[:, :Hd] = feats
    wa = np.zeros((A, Hp), np.float32); wa[:, :Hd] = d["weight"]
    fd, wad, bad = _dev(f), _dev(wa), _dev(d["bias"])
    wc, bc = torch.zeros(Hp, device=gpu), torch.zeros(1, device=gpu)
    noise = _dev(d["exp_noise"])
    val = torch.empty(N, device=gpu); act = torch.empty(N, dtype=torch.int64, device=gpu)
    lp = torch.empty(N, device=gpu); ent = torch.empty(N, device=gpu)
    Hh.call("ppo_heads_act", fd.data_ptr(), None, N, Hp, wc.data_ptr(), bc.data_ptr(), wad.data_ptr(), bad.data_ptr(), A,
            noise.data_ptr(), 0, 0, 0, None, val.data_ptr(), act.data_ptr(), lp.data_ptr(), ent.data_ptr(), _s())
    assert np.array_equal(act.cpu().numpy(), d["action"][:, 0])                  # bit-exact sampling
    np.testing.assert_allclose(lp.cpu().numpy(), d["log_probs"][:, 0], atol=2e-6)
    np.testing.assert_allclose(ent.cpu().numpy(), d["entropy"], atol=2e-6)
    Hh.call("ppo_heads_act", fd.data_ptr(), None, N, Hp, wc.data_ptr(), bc.data_ptr(), wad.data_ptr(), bad.data_ptr(), A,
            None, 0, 0, 1, None, val.data_ptr(), act.data_ptr(), lp.data_ptr(), ent.data_ptr(), _s())
    assert np.array_equal(act.cpu().numpy(), d["mode"][:, 0])


def test_device_sampling_distribution(gpu):
    """device RNG mode: empirical action frequencies match probs (chi-square-ish)."""
    Hh = _hip()
    N, Hp, A = 200000, 64, 8
    f = torch.zeros(N, Hp, device=gpu); f[:, 0] = 1.0
    wa = torch.zeros(A, Hp, device=gpu); wa[:, 0] = torch.linspace(-1, 1.5, A, device=gpu)
    ba = torch.zeros(A, device=gpu)
    wc, bc = torch.zeros(Hp, device=gpu), torch.zeros(1, device=gpu)
    act = torch.empty(N, dtype=torch.int64, device=gpu)
    Hh.call("ppo_heads_act", f.data_ptr(), None, N, Hp, wc.data_ptr(), bc.data_ptr(), wa.data_ptr(), ba.data_ptr(), A,
            None, 1234, 1, 0, None, None, act.data_ptr(), None, None, _s())
    freq = np.bincount(act.cpu().numpy(), minlength=A) / N
    p = torch.softmax(torch.linspace(-1, 1.5, A), 0).numpy()
    assert np.abs(freq - p).max() < 0.005


# --------------------------------------------------------------- optimizer (K17/K18)
def test_clip_adam_golden(gpu):
    Hh = _hip()
    d = golden("adam_clip.npz")
    n = d["init"].size
    p = _dev(d["init"])
    m = torch.zeros(n, device=gpu); v = torch.zeros(n, device=gpu)
    parts = torch.zeros(Hh.call("ppo_grad_partials_count", n), dtype=torch.float64, device=gpu)
    nrm = torch.zeros(1, dtype=torch.float64, device=gpu)
    for k in range(d["grads"].shape[0]):
        g = _dev(d["grads"][k])
        Hh.call("ppo_grad_sumsq", g.data_ptr(), n, 1.0, parts.data_ptr(), _s())
        Hh.call("ppo_clip_adam", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, parts.data_ptr(), 1.0,
                float(d["max_norm"][0]), float(d["lr"][0]), 0.9, 0.999, float(d["eps"][0]), k + 1, nrm.data_ptr(),
                _s())
        np.testing.assert_allclose(nrm.item(), d["total_norms"][k], rtol=1e-6)
        np.testing.assert_allclose(g.cpu().numpy(), d["clipped"][k], rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(p.cpu().numpy(), d["after"][k], rtol=0, atol=1e-6)


# ------------------------------------------------------------------ whole iteration
def test_full_iteration_replays_reference(gpu):
    """The reference iteration recorded in cnn_update.npz, replayed through the
    drop-in API: same init (same seed + construction), same host sampling draws,
    same randperms -> bit-exact actions, returns within 1e-5, losses within 1e-4
    relative, final parameters within 2e-5 absolute (lr 1e-3 steps)."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("cnn_update.npz")
    hidden, N, T, E, Mb = (int(x) for x in d["meta"])
    torch.set_num_threads(1)   # as T/run.py:55 (orthogonal_ init is thread-count sensitive)
    torch.manual_seed(1)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase,
                   base_kwargs={"recurrent": False, "hidden_size": hidden}, vector_obs_len=0)
    # identical construction + init is asserted on the container's CPU
    # (tests/test_host_cpu.py); orthogonal_'s LAPACK QR may round differently
    # on another host CPU, so start from the reference's recorded parameters.
    with torch.no_grad():
        flat = torch.from_numpy(d["init_params"])
        off = 0
        for p in pol.parameters():
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
    pol.to(gpu)
    agent = PPO(pol, 0.1, E, Mb, 0.5, 0.001, lr=float(d["lr"][0]), eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), pol.recurrent_hidden_state_size,
                        obs_dtype=torch.uint8, device=gpu)
    st.obs.copy_(_dev(d["obs_u8"]))
    M.set_sampling_mode("host")
    try:
        for step in range(T):
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                  st.masks[step])
            st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, _dev(d["rewards"][step]),
                      _dev(d["masks"][step]), torch.ones(N, 1, device=gpu))
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, False)
        losses = agent.update(st)
    finally:
        M.set_sampling_mode("device")
    assert np.array_equal(st.actions.cpu().numpy(), d["actions"])
    np.testing.assert_allclose(st.action_log_probs.cpu().numpy(), d["action_log_probs"], atol=1e-5)
    np.testing.assert_allclose(st.returns.cpu().numpy(), d["returns"], atol=1e-5)
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4, atol=1e-6)
    final = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu().numpy()
    np.testing.assert_allclose(final, d["final_params"], rtol=0, atol=2e-5)
    st.after_update()
    assert torch.equal(st.obs[0], st.obs[-1])


def test_full_size_forward_vs_oracle(gpu):
    """c3 network (H=512) on 4096 lanes: value/log-prob through Policy.act
    (deterministic) vs the float64 oracle — max abs err 1e-4."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import Discrete
    torch.manual_seed(5)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": False})
    init = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy()
    pol.to(gpu)
    N = 4096
    g = torch.Generator().manual_seed(6)
    obs = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, generator=g)
    v, a, lp, _ = pol.act(obs.cuda(), None, None, None, deterministic=True)
    sub = np.arange(0, N, 64)
    p = O.unflatten(init, O.cnn_param_shapes(512))
    value, logits, _ = O.cnn_forward(p, O.decode_obs(obs.numpy()[sub]))
    c = O.categorical(logits, deterministic=True)
    np.testing.assert_allclose(v.cpu().numpy()[sub, 0], value, atol=1e-4)
    np.testing.assert_allclose(lp.cpu().numpy()[sub, 0], c["log_prob"], atol=1e-4)


# ------------------------------------------------------------------ GRU (K12)
def _load_flat(pol, flat):
    with torch.no_grad():
        off = 0
        for p in pol.parameters():
            p.copy_(torch.from_numpy(np.ascontiguousarray(flat[off:off + p.numel()])).view_as(p))
            off += p.numel()


def test_gru_golden_evaluate_and_step(gpu):
    """Recurrent CNNBase + vector obs (T/model.py:89-166,192-199) on the reference's
    recorded sequence: values / log-probs / entropy / final hidden within 2e-5,
    and the single-step act path (model.py:112-115)."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("gru_eval.npz")
    hidden, V, N, T = (int(x) for x in d["meta"])
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": hidden},
                   vector_obs_len=V)
    _load_flat(pol, d["params"])
    pol.to(gpu)
    obs = _dev(d["obs_u8"].reshape(T * N, 4, 84, 84))
    vec = _dev(d["vector_obs"].reshape(T * N, V))
    masks = _dev(d["masks"].reshape(T * N, 1))
    h0 = _dev(d["h0"])
    acts = _dev(d["actions"])
    value, logp, ent, hT = pol.evaluate_actions(obs, vec, h0, masks, acts)
    np.testing.assert_allclose(value.cpu().numpy(), d["values"], atol=2e-5)
    np.testing.assert_allclose(logp.cpu().numpy(), d["log_probs"], atol=2e-5)
    np.testing.assert_allclose(ent.item(), d["entropy"][0], atol=2e-5)
    np.testing.assert_allclose(hT.cpu().numpy(), d["hT"], atol=2e-5)
    v1, a1, lp1, h1 = pol.act(obs[:N], vec[:N], h0, _dev(d["masks"][0]), deterministic=True)
    np.testing.assert_allclose(v1.cpu().numpy(), d["step_value"], atol=2e-5)
    np.testing.assert_allclose(h1.cpu().numpy(), d["step_h"], atol=2e-5)


@pytest.mark.parametrize("H,V", [(64, 14), (256, 14)])
def test_recurrent_minibatch_grads_vs_oracle(gpu, H, V):
    """One recurrent_generator minibatch through the fused path (trunk, vector-obs
    concat, GRU over T with masks, heads/loss, BPTT, all wgrads) vs the oracle's
    float64 analytic gradients: max |err| <= 2e-5 * max|grad| per tensor."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo.ppo import FlatAdam
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    torch.manual_seed(H)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
                   vector_obs_len=V)
    with torch.no_grad():
        pol.dist.linear.weight.mul_(50.0)
        pol.base.critic_linear.weight.mul_(3.0)
        pol.base.gru.bias_ih_l0.uniform_(-0.3, 0.3)
        pol.base.gru.bias_hh_l0.uniform_(-0.3, 0.3)
    init = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy().astype(np.float64)
    pol.to(gpu)
    eng = pol.hip_engine()
    T, N = 5, 6
    st = RolloutStorage(T, N, (4, 84, 84), [V], Discrete(8), H, obs_dtype=torch.uint8, device=gpu)
    g = torch.Generator().manual_seed(H + 1)
    st.obs.copy_(torch.randint(0, 256, st.obs.shape, dtype=torch.uint8, generator=g).to(gpu))
    st.vector_obs.copy_(torch.rand(st.vector_obs.shape, generator=g).to(gpu))
    st.recurrent_hidden_states.copy_(torch.randn(st.recurrent_hidden_states.shape, generator=g).to(gpu) * 0.5)
    st.masks.copy_((torch.rand(st.masks.shape, generator=g) > 0.3).float().to(gpu))
    st.actions.copy_(torch.randint(0, 8, st.actions.shape, generator=g).to(gpu))
    st.action_log_probs.copy_((torch.log(torch.rand(st.action_log_probs.shape, generator=g)) * 0.3 - 2.0).to(gpu))
    st.value_preds.copy_(torch.randn(st.value_preds.shape, generator=g).to(gpu) * 0.1)
    st.returns.copy_(torch.randn(st.returns.shape, generator=g).to(gpu))
    adv = torch.randn(T, N, generator=g).to(gpu)
    envs = torch.tensor([4, 0, 3], dtype=torch.int64)
    hp = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.01, "use_clipped_value_loss": True}
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)   # 3 losses + bad-action count
    opt = FlatAdam(pol.parameters(), lr=0.0, eps=1e-5, max_grad_norm=None)
    eng.train_minibatch_rec(st, adv, envs.to(gpu), hp, loss, opt)
    torch.cuda.synchronize()
    shapes = O.cnn_param_shapes(H, recurrent=True, vector_obs_len=V)
    p = O.unflatten(init, shapes)
    e = envs.numpy()
    rows = (np.arange(T)[:, None] * N + e[None, :]).reshape(-1)
    obs = st.obs[:-1].reshape(T * N, 4, 84, 84).cpu().numpy()[rows]
    vec = st.vector_obs[:-1].reshape(T * N, V).cpu().numpy()[rows]
    h0 = st.recurrent_hidden_states[0].cpu().numpy()[e]
    masks = st.masks[:-1, :, 0].cpu().numpy()[:, e]
    value, logits, cache = O.recurrent_forward(p, O.decode_obs(obs), vec, h0, masks)
    f = lambda t: t.reshape(-1).cpu().numpy()[rows]  # noqa: E731
    lg = O.loss_head_grads(value, logits, f(st.actions), f(st.action_log_probs), f(adv),
                           st.value_preds[:-1].reshape(-1).cpu().numpy()[rows],
                           st.returns[:-1].reshape(-1).cpu().numpy()[rows], 0.1, 0.5, 0.01)
    grads = O.recurrent_backward(p, cache, lg["g_value"], lg["g_logits"])
    got = O.unflatten(eng.grad.cpu().numpy(), shapes)
    for name, _ in shapes:
        ref = grads[name]
        err = np.abs(got[name] - ref).max()
        assert err <= 2e-5 * max(np.abs(ref).max(), 1e-3), (name, err, np.abs(ref).max())
    np.testing.assert_allclose(loss.cpu().numpy()[:3], [lg["value_loss"], lg["action_loss"], lg["entropy"]],
                               rtol=2e-5, atol=1e-6)


def test_recurrent_ppo_iteration_runs(gpu):
    """c5-shaped plumbing at small scale: rollout with hidden state carry, GAE,
    recurrent PPO.update (BPTT), after_update — finite losses, parameters move."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    torch.manual_seed(2)
    N, T, V, H = 16, 8, 14, 64
    env = SyntheticVecEnv(N, seed=5, p_done=0.2, device=gpu)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
                   vector_obs_len=V)
    pol.to(gpu)
    agent = PPO(pol, 0.1, 2, 4, 0.5, 0.001, lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [V], env.action_space, H, obs_dtype=torch.uint8, device=gpu)
    env.reset_into(st.obs[0])
    before = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    for step in range(T):
        v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step], st.masks[step])
        r, m, bm = env.step_into(st.obs[step + 1], a)
        st.insert(st.obs[step + 1], torch.rand(N, V, device=gpu), h, a, lp, v, r, m, bm)
    nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
    st.compute_returns(nv, True, 0.99, 0.95, False)
    losses = agent.update(st)
    st.after_update()
    after = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    assert all(np.isfinite(losses))
    assert (after - before).abs().max().item() > 1e-5
    assert torch.equal(st.recurrent_hidden_states[0], st.recurrent_hidden_states[-1])


def test_recurrent_iteration_replays_reference(gpu):
    """The reference's recurrent iteration recorded in gru_update.npz (T/ GRU +
    vector obs, hidden 32, V 14, 8 envs x 16 steps, masks with zeros, a carried
    initial hidden state; PPO.update over recurrent_generator, E = 2, M = 2)
    replayed through the drop-in API in host-sampling mode: actions bit-exact,
    log-probs / values / returns / the carried hidden state within 1e-5, the first
    minibatch's gradient (BPTT through the masked sequences) within 1e-5 of each
    tensor's max |g|, every minibatch's losses within 1e-4 relative, the final
    parameters within 2e-5 (T/a2c_ppo_acktr/storage.py:162-223, model.py:111-166,
    algo/ppo.py:43-96)."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("gru_update.npz")
    hidden, V, N, T, E, Mb = (int(x) for x in d["meta"])
    clip, vcoef, ecoef = (float(x) for x in d["coefs"])
    torch.set_num_threads(1)
    torch.manual_seed(31)   # the generator's seed: construction consumes the same draws as the reference's
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": hidden},
                   vector_obs_len=V)
    _load_flat(pol, d["init_params"])
    pol.to(gpu)
    agent = PPO(pol, clip, E, Mb, vcoef, ecoef, lr=float(d["lr"][0]), eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [V], Discrete(8), pol.recurrent_hidden_state_size,
                        obs_dtype=torch.uint8, device=gpu)
    st.obs.copy_(_dev(d["obs_u8"]))
    st.vector_obs.copy_(_dev(d["vector_obs"]))
    st.recurrent_hidden_states[0].copy_(_dev(d["h0"]))
    st.masks[0].copy_(_dev(d["masks0"]))
    eng = pol.hip_engine()
    grads, accs = [], []
    orig_step = agent.optimizer._step_flat

    def step_capture(e):
        grads.append(e.grad.clone())          # before clip + Adam (the reference's clip_grad_norm_ input)
        accs.append(agent._loss_acc[:3].clone())
        return orig_step(e)

    agent.optimizer._step_flat = step_capture
    M.set_sampling_mode("host")
    try:
        for step in range(T):
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                  st.masks[step])
            st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, _dev(d["rewards"][step]),
                      _dev(d["masks"][step]), torch.ones(N, 1, device=gpu))
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, False)
        losses = agent.update(st)
    finally:
        M.set_sampling_mode("device")
        agent.optimizer._step_flat = orig_step
    assert eng is pol.hip_engine()
    assert np.array_equal(st.actions.cpu().numpy(), d["actions"])
    np.testing.assert_allclose(st.action_log_probs.cpu().numpy(), d["action_log_probs"], atol=1e-5)
    np.testing.assert_allclose(st.value_preds[:T].cpu().numpy(), d["values"], atol=1e-5)
    np.testing.assert_allclose(st.recurrent_hidden_states[-1].cpu().numpy(), d["hidden_T"], atol=1e-5)
    np.testing.assert_allclose(st.returns.cpu().numpy(), d["returns"], atol=1e-5)
    assert len(grads) == E * Mb
    shapes = O.cnn_param_shapes(hidden, recurrent=True, vector_obs_len=V)
    got, ref = O.unflatten(grads[0].cpu().numpy(), shapes), O.unflatten(d["mb0_preclip_grad"], shapes)
    for name, _ in shapes:
        err = np.abs(got[name] - ref[name]).max()
        assert err <= 1e-5 * max(np.abs(ref[name]).max(), 1e-6), (name, err, np.abs(ref[name]).max())
    acc = torch.stack(accs + [agent._loss_acc[:3].clone()]).cpu().numpy()
    # the loss accumulator before each step holds the minibatches up to and including it
    mb = np.diff(np.concatenate([np.zeros((1, 3)), acc[:-1]], 0), axis=0)
    np.testing.assert_allclose(mb, d["mb_losses"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4, atol=1e-6)
    final = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu().numpy()
    np.testing.assert_allclose(final, d["final_params"], rtol=0, atol=2e-5)


# ------------------------------------------------------------- MLPBase (c1)
def _mlp_policy(gpu, I, V, H, A, seed):
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import Discrete
    torch.manual_seed(seed)
    return M.Policy((I,), Discrete(A), base=M.MLPBase, base_kwargs={"recurrent": False, "hidden_size": H},
                    vector_obs_len=V)


def test_mlp_golden_evaluate(gpu):
    """MLPBase + Categorical(64, 2) with the reference's parameters (mlp.npz):
    value, log-prob and entropy through Policy.evaluate_actions within 1e-5."""
    d = golden("mlp.npz")
    pol = _mlp_policy(gpu, 4, 0, 64, 2, 0)
    _load_flat(pol, np.concatenate([d["base_params"], d["head_params"]]))
    pol.to(gpu)
    x = _dev(d["x"])
    B = x.shape[0]
    for a in (0, 1):
        act = torch.full((B, 1), a, dtype=torch.int64, device=gpu)
        v, lp, ent, _ = pol.evaluate_actions(x, None, None, None, act)
        np.testing.assert_allclose(v.cpu().numpy(), d["value"], atol=1e-5)
        np.testing.assert_allclose(lp.cpu().numpy()[:, 0], d["norm_logits"][:, a], atol=1e-5)
        np.testing.assert_allclose(float(ent), d["entropy"].mean(), atol=1e-5)
    v2 = pol.get_value(x, None, None, None)
    np.testing.assert_allclose(v2.cpu().numpy(), d["value"], atol=1e-5)
    _, a, lp, _ = pol.act(x, None, None, None, deterministic=True)
    assert np.array_equal(a.cpu().numpy()[:, 0], d["norm_logits"].argmax(1))


@pytest.mark.parametrize("I,V,H,A,B", [(4, 0, 64, 2, 256), (5, 3, 128, 6, 37)])
def test_mlp_minibatch_grads_vs_oracle(gpu, I, V, H, A, B):
    """One feed-forward minibatch of an MLPBase policy (input gather + vector-obs
    concat + padding, tanh towers, heads/loss, every dgrad/wgrad) vs the oracle's
    float64 analytic gradients: max |err| <= 1e-5 * max|grad| per tensor."""
    from a2c_ppo_acktr.algo.ppo import FlatAdam
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    pol = _mlp_policy(gpu, I, V, H, A, B)
    with torch.no_grad():
        pol.dist.linear.weight.mul_(20.0)
        pol.base.critic_linear.weight.mul_(3.0)
    init = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy().astype(np.float64)
    pol.to(gpu)
    eng = pol.hip_engine()
    T, N = 4, (B + 1) // 2
    st = RolloutStorage(T, N, (I,), [V], Discrete(A), 1, device=gpu)
    g = torch.Generator().manual_seed(B + 1)
    st.obs.copy_(torch.randn(st.obs.shape, generator=g).to(gpu))
    if V:
        st.vector_obs.copy_(torch.rand(st.vector_obs.shape, generator=g).to(gpu))
    st.actions.copy_(torch.randint(0, A, st.actions.shape, generator=g).to(gpu))
    st.action_log_probs.copy_((torch.log(torch.rand(st.action_log_probs.shape, generator=g)) * 0.3 - 1.0).to(gpu))
    st.value_preds.copy_(torch.randn(st.value_preds.shape, generator=g).to(gpu) * 0.1)
    st.returns.copy_(torch.randn(st.returns.shape, generator=g).to(gpu))
    adv = torch.randn(T, N, generator=g).to(gpu)
    idx = torch.randperm(T * N, generator=g)[:B].to(gpu)
    hp = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.01, "use_clipped_value_loss": True}
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)   # 3 losses + bad-action count
    opt = FlatAdam(pol.parameters(), lr=0.0, eps=1e-5, max_grad_norm=None)
    eng.train_minibatch(st, adv, idx, hp, loss, opt)
    torch.cuda.synchronize()
    shapes = O.mlp_param_shapes(I + V, H, A)
    p = O.unflatten(init, shapes)
    ii = idx.cpu().numpy()
    x = st.obs[:-1].reshape(T * N, I).cpu().numpy()[ii]
    if V:
        x = np.concatenate([x, st.vector_obs[:-1].reshape(T * N, V).cpu().numpy()[ii]], 1)
    value, logits, cache = O.mlp_forward(p, x.astype(np.float64))
    f = lambda t: t.reshape(-1).cpu().numpy()[ii]  # noqa: E731
    lg = O.loss_head_grads(value, logits, f(st.actions), f(st.action_log_probs), f(adv),
                           st.value_preds[:-1].reshape(-1).cpu().numpy()[ii],
                           st.returns[:-1].reshape(-1).cpu().numpy()[ii], 0.1, 0.5, 0.01)
    grads = O.mlp_backward(p, cache, lg["g_value"], lg["g_logits"])
    got = O.unflatten(eng.grad.cpu().numpy(), shapes)
    for name, _ in shapes:
        ref = grads[name]
        err = np.abs(got[name] - ref).max()
        assert err <= 1e-5 * max(np.abs(ref).max(), 1e-3), (name, err, np.abs(ref).max())
    np.testing.assert_allclose(loss.cpu().numpy()[:3], [lg["value_loss"], lg["action_loss"], lg["entropy"]],
                               rtol=2e-5, atol=1e-6)


def test_cartpole_env_vs_oracle(gpu):
    """CartPoleVecEnv (one fp32 kernel) vs the numpy restatement, step by step
    from the same state: observations within 1e-5, reward/mask/bad_mask/episode
    length and every counter-RNG reset exact."""
    from a2c_ppo_acktr.synthetic import CartPoleVecEnv
    N = 512
    env = CartPoleVecEnv(N, seed=11, max_steps=60, device=gpu)
    obs = torch.empty(N, 4, device=gpu)
    env.reset_into(obs)
    st0, k0 = O.cartpole_step(np.zeros((N, 4)), np.zeros(N), None, 11, 0)[:2]
    np.testing.assert_array_equal(env.state.cpu().numpy(), st0)
    g = torch.Generator().manual_seed(0)
    ended = 0
    for c in range(1, 150):
        st, k = env.state.cpu().numpy(), env.steps.cpu().numpy()
        a = torch.randint(0, 2, (N, 1), generator=g)
        r, m, bm = env.step_into(obs, a.to(gpu))
        est, ek, eobs, er, em, ebm, eep = O.cartpole_step(st, k, a.numpy(), 11, c, max_steps=60)
        np.testing.assert_array_equal(m.cpu().numpy()[:, 0], em)
        np.testing.assert_array_equal(bm.cpu().numpy()[:, 0], ebm)
        np.testing.assert_array_equal(r.cpu().numpy()[:, 0], er)
        np.testing.assert_array_equal(env.ep_len.cpu().numpy(), eep)
        np.testing.assert_array_equal(env.steps.cpu().numpy(), ek)
        np.testing.assert_allclose(obs.cpu().numpy(), eobs, rtol=1e-5, atol=1e-6)
        ended += int((em == 0).sum())
    assert ended > N   # plenty of terminations and TimeLimit truncations exercised


@pytest.mark.parametrize("N,Mb,iters", [(16, 4, 60), (8, 32, 60)])
def test_ppo_learns_cartpole(gpu, N, Mb, iters):
    """c1 end to end (MLPBase hidden 64, GPU CartPole, GAE, PPO.update): the
    mean finished-episode length must rise well above a random policy's ~22.
    (8, 32) is c1's own shape (8 envs x 128 steps, 4 epochs, 32
    minibatches of 32 samples)."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import CartPoleVecEnv
    torch.manual_seed(0)
    T = 128
    env = CartPoleVecEnv(N, seed=3, device=gpu)
    pol = M.Policy(env.obs_shape, env.action_space, base=M.MLPBase, base_kwargs={"recurrent": False})
    pol.to(gpu)
    agent = PPO(pol, 0.2, 4, Mb, 0.5, 0.0, lr=2.5e-3, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, env.obs_shape, [0], env.action_space, 1, device=gpu)
    env.reset_into(st.obs[0])
    hist = []
    for it in range(iters):
        tot = torch.zeros(2, device=gpu)
        for step in range(T):
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                  st.masks[step])
            r, m, bm = env.step_into(st.obs[step + 1], a)
            tot[0] += env.ep_len.sum()
            tot[1] += (env.ep_len > 0).sum()
            st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, r, m, bm)
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, True)
        losses = agent.update(st)
        st.after_update()
        t = tot.cpu().numpy()
        hist.append(t[0] / max(t[1], 1))
        assert all(np.isfinite(losses))
    early, late = np.mean(hist[:3]), np.mean(hist[-5:])
    print("cartpole mean episode length", early, "->", late)
    assert early < 40 and late > 150, hist


def test_packed_weight_planes_exact(gpu):
    """ppo_pack_weights writes, after every packed fp32 segment, its exact bf16
    split (hi, mid, lo planes): hi + mid + lo reproduces each fp32 value bit for bit."""
    Hh = _hip()
    H = 64
    g = torch.Generator().manual_seed(3)
    w2 = (torch.randn(64, 32, 4, 4, generator=g) * 0.1).cuda()
    w3 = (torch.randn(32, 64, 3, 3, generator=g) * 0.1).cuda()
    w4 = (torch.randn(H, 1568, generator=g) * 0.02).cuda()
    packed = torch.zeros(Hh.call("ppo_packed_weights_size", H), device=gpu)
    offs = torch.zeros(6, dtype=torch.int64)
    Hh.call("ppo_packed_offsets", H, offs.data_ptr())
    Hh.call("ppo_pack_weights", w2.data_ptr(), w3.data_ptr(), w4.data_ptr(), H, packed.data_ptr(), _s())
    torch.cuda.synchronize()
    buf = packed.cpu().numpy()
    sizes = [64 * 512, 32 * 576, H * 1568, H * 1568, 64 * 288, 4 * 32 * 256]
    for o, n in zip(offs.tolist(), sizes):
        seg = buf[o:o + n]
        planes = buf[o + n:o + n + 3 * n // 2].view(np.uint16).astype(np.uint32)
        parts = [(planes[i * n:(i + 1) * n] << 16).view(np.float32).astype(np.float64) for i in range(3)]
        assert np.array_equal(parts[0] + parts[1] + parts[2], seg.astype(np.float64))
    # and the packed values themselves are the torch weights, reordered (spot check of W4p)
    w4p = buf[offs[2]:offs[2] + H * 1568].reshape(H, 49, 32)   # [n][p][c]
    ref = w4.cpu().numpy().reshape(H, 32, 49).transpose(0, 2, 1)
    assert np.array_equal(w4p, ref)


def _packed(gpu, H, seed):
    Hh = _hip()
    g = torch.Generator().manual_seed(seed)
    w = {"w2": torch.randn(64, 32, 4, 4, generator=g) * 0.05, "w3": torch.randn(32, 64, 3, 3, generator=g) * 0.05,
         "w4": torch.randn(H, 1568, generator=g) * 0.02}
    d = {k: v.cuda() for k, v in w.items()}
    packed = torch.zeros(Hh.call("ppo_packed_weights_size", H), device=gpu)
    offs = torch.zeros(6, dtype=torch.int64)
    Hh.call("ppo_packed_offsets", H, offs.data_ptr())
    Hh.call("ppo_pack_weights", d["w2"].data_ptr(), d["w3"].data_ptr(), d["w4"].data_ptr(), H, packed.data_ptr(),
            _s())
    return w, packed, [packed.data_ptr() + 4 * int(o) for o in offs]


def test_conv2_dgrad_vs_torch(gpu):
    """conv2 dgrad (phase-merged GEMM, 4x4 stride 2 transposed conv 9x9 -> 20x20
    with the conv1 ReLU mask) on the image-resident exact split-bf16 kernel vs torch float64:
    max |err| <= 1e-5 * max |ref| (fp32 arithmetic, summation order differs).
    B = 300 images > the persistent grid, so blocks walk several images."""
    Hh = _hip()
    B = 300
    w, packed, pk = _packed(gpu, 64, 11)
    g = torch.Generator().manual_seed(12)
    dz2 = torch.randn(B, 9, 9, 64, generator=g)
    a1 = torch.randn(B, 20, 20, 32, generator=g)
    dz1 = torch.full((B, 20, 20, 32), float("nan"), device=gpu)
    dz2_d, a1_d = dz2.cuda(), a1.cuda()
    Hh.call("ppo_conv2_dgrad", dz2_d.data_ptr(), B, pk[5], a1_d.data_ptr(), dz1.data_ptr(), _s())
    torch.cuda.synchronize()
    ref = F.conv_transpose2d(dz2.double().permute(0, 3, 1, 2), w["w2"].double(), stride=2).permute(0, 2, 3, 1)
    ref = torch.where(a1 > 0, ref, torch.zeros((), dtype=torch.float64))
    err = (dz1.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


@pytest.mark.parametrize("conv1_variant", [0, 9])
def test_conv1_mask_bits_and_conv2_dgrad_bits(gpu, conv1_variant):
    """ppo_conv1_fwd_mask (fused ballot epilogue: variant 0; conv + relu_bits
    kernel: variant 9) writes bit c of word p = (a1[p][c] > 0) of its own fp32
    output, bit-exactly, with a1 identical to ppo_conv1_fwd's; conv2 dgrad fed
    those bits (ppo_conv2_dgrad_bits) equals the fp32-mask kernel bit for bit.
    B = 300 > the persistent grid, gathered storage rows."""
    Hh = _hip()
    B = 300
    g = torch.Generator().manual_seed(31)
    obs = torch.randint(0, 256, (B + 5, 4, 84, 84), dtype=torch.uint8, generator=g).cuda()
    idx = torch.randperm(B + 5, generator=g)[:B].cuda()
    w1 = (torch.randn(32, 256, generator=g) * 0.05).cuda()
    b1 = (torch.randn(32, generator=g) * 0.2).cuda()   # a mix of live and dead units
    a1 = torch.full((B, 20, 20, 32), float("nan"), device=gpu)
    a1m = torch.full_like(a1, float("nan"))
    bits = torch.zeros(B * 400, dtype=torch.int32, device=gpu)
    old_tune = Hh.call("ppo_tune_get", b"conv1_fwd")
    Hh.call("ppo_tune_set", b"conv1_fwd", conv1_variant)
    try:
        Hh.call("ppo_conv1_fwd", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
                a1.data_ptr(), _s())
        Hh.call("ppo_conv1_fwd_mask", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
                a1m.data_ptr(), bits.data_ptr(), _s())
        torch.cuda.synchronize()
    finally:
        Hh.call("ppo_tune_set", b"conv1_fwd", old_tune)
    assert torch.equal(a1, a1m)
    live = (a1 > 0).reshape(B * 400, 32).cpu().to(torch.int64)
    want = (live << torch.arange(32, dtype=torch.int64)).sum(1)
    got = bits.cpu().to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(got, want)
    assert 0.2 < live.float().mean().item() < 0.8
    _, packed, pk = _packed(gpu, 64, 32)   # keep the packed buffer alive
    dz2 = torch.randn(B, 9, 9, 64, generator=g).cuda()
    d_ref = torch.full_like(a1, float("nan"))
    d_bits = torch.full_like(a1, float("nan"))
    Hh.call("ppo_conv2_dgrad", dz2.data_ptr(), B, pk[5], a1.data_ptr(), d_ref.data_ptr(), _s())
    assert Hh.call("ppo_conv2_dgrad_bits_ok") == 1
    Hh.call("ppo_conv2_dgrad_bits", dz2.data_ptr(), B, pk[5], bits.data_ptr(), d_bits.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(d_ref, d_bits)


def test_conv2_mask_bits_and_conv3_dgrad_bits(gpu):
    """ppo_conv2_fwd_mask (fused ballot epilogue) writes bit c of word p = (a2[p][c] > 0) of its own fp32
    output, with a2 identical to ppo_conv2_fwd's; conv3 dgrad fed those bits
    (ppo_conv3_dgrad_bits) equals the fp32-mask kernel bit for bit.  B = 300."""
    Hh = _hip()
    B = 300
    _, packed, pk = _packed(gpu, 64, 41)   # keep the packed buffer alive
    g = torch.Generator().manual_seed(42)
    a1 = torch.relu(torch.randn(B, 20, 20, 32, generator=g)).cuda()
    b2 = (torch.randn(64, generator=g) * 0.1).cuda()
    a2 = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
    a2m = torch.full_like(a2, float("nan"))
    bits = torch.zeros(B * 81, dtype=torch.int64, device=gpu)
    Hh.call("ppo_conv2_fwd", a1.data_ptr(), B, pk[0], b2.data_ptr(), a2.data_ptr(), _s())
    Hh.call("ppo_conv2_fwd_mask", a1.data_ptr(), B, pk[0], b2.data_ptr(), a2m.data_ptr(), bits.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(a2, a2m)
    live = (a2 > 0).reshape(B * 81, 64).cpu()
    got = bits.cpu()
    for h in range(2):   # 32-bit halves (int64 arithmetic cannot hold bit 63 unsigned)
        want = (live[:, 32 * h:32 * h + 32].to(torch.int64) << torch.arange(32, dtype=torch.int64)).sum(1)
        assert torch.equal((got >> (32 * h)) & 0xFFFFFFFF, want)
    assert 0.2 < live.float().mean().item() < 0.8
    dz3 = torch.randn(B, 7, 7, 32, generator=g).cuda()
    d_ref = torch.full_like(a2, float("nan"))
    d_bits = torch.full_like(a2, float("nan"))
    Hh.call("ppo_conv3_dgrad", dz3.data_ptr(), B, pk[4], a2.data_ptr(), d_ref.data_ptr(), _s())
    assert Hh.call("ppo_conv3_dgrad_bits_ok") == 1
    Hh.call("ppo_conv3_dgrad_bits", dz3.data_ptr(), B, pk[4], bits.data_ptr(), d_bits.data_ptr(), _s())
    torch.cuda.synchronize()
    assert torch.equal(d_ref, d_bits)


@pytest.mark.parametrize("B", [5, 300, 4096])
@pytest.mark.parametrize("products", [6, 1, 9])
def test_trunk_fwd_equals_three_launches(gpu, B, products):
    """ppo_trunk_fwd (conv1 -> conv2 -> conv3 as three phases of one persistent
    launch, the rollout's trunk) writes a1, a2, a3 bit-identical to ppo_conv1_fwd,
    ppo_conv2_fwd and ppo_conv3_fwd, rows gathered out of order: B < the grid
    (blocks without images), blocks walking 2 images, and the rollout's 4,096 (16
    per block); every product count.  The masked form (both mask buffers) equals
    ppo_conv1_fwd_mask / ppo_conv2_fwd_mask."""
    Hh = _hip()
    _, packed, pk = _packed(gpu, 64, 51)
    g = torch.Generator().manual_seed(52 + B)
    rows = B + 64
    obs = torch.randint(0, 256, (rows, 4, 84, 84), dtype=torch.uint8, generator=g).cuda()
    idx = torch.randperm(rows, generator=g)[:B].contiguous().cuda()
    w1 = (torch.randn(32, 4, 8, 8, generator=g) * 0.05).cuda()
    b1, b2, b3 = [(torch.randn(n, generator=g) * 0.1).cuda() for n in (32, 64, 32)]
    def bufs():
        return [torch.full((B * n,), float("nan"), device=gpu) for n in (400 * 32, 81 * 64, 49 * 32)]
    old = Hh.call("ppo_tune_get", b"products")
    try:
        Hh.call("ppo_tune_set", b"products", products)
        r1, r2, r3 = bufs()
        Hh.call("ppo_conv1_fwd", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
                r1.data_ptr(), _s())
        Hh.call("ppo_conv2_fwd", r1.data_ptr(), B, pk[0], b2.data_ptr(), r2.data_ptr(), _s())
        Hh.call("ppo_conv3_fwd", r2.data_ptr(), B, pk[1], b3.data_ptr(), r3.data_ptr(), _s())
        t1, t2, t3 = bufs()
        Hh.call("ppo_trunk_fwd", obs.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(), b1.data_ptr(), t1.data_ptr(),
                None, pk[0], b2.data_ptr(), t2.data_ptr(), None, pk[1], b3.data_ptr(), t3.data_ptr(), _s())
        m1 = torch.zeros(B * 400, dtype=torch.int32, device=gpu)
        m2 = torch.zeros(B * 81, dtype=torch.int64, device=gpu)
        q1 = torch.zeros_like(m1)
        q2 = torch.zeros_like(m2)
        u1, u2, u3 = bufs()
        Hh.call("ppo_trunk_fwd", obs.data_ptr(), idx.data_ptr(), 0, B, w1.data_ptr(), b1.data_ptr(), u1.data_ptr(),
                m1.data_ptr(), pk[0], b2.data_ptr(), u2.data_ptr(), m2.data_ptr(), pk[1], b3.data_ptr(),
                u3.data_ptr(), _s())
        v1, v2 = bufs()[:2]
        Hh.call("ppo_conv1_fwd_mask", obs.data_ptr(), 1, idx.data_ptr(), 0, 4, B, w1.data_ptr(), b1.data_ptr(),
                v1.data_ptr(), q1.data_ptr(), _s())
        Hh.call("ppo_conv2_fwd_mask", v1.data_ptr(), B, pk[0], b2.data_ptr(), v2.data_ptr(), q2.data_ptr(), _s())
        torch.cuda.synchronize()
    finally:
        Hh.call("ppo_tune_set", b"products", old)
    for a, b in ((r1, t1), (r2, t2), (r3, t3), (r1, u1), (r2, u2), (r3, u3)):
        assert torch.equal(a, b)
    assert torch.equal(m1, q1) and torch.equal(m2, q2)
    assert 0.2 < (r3 > 0).float().mean().item() < 0.8


@pytest.mark.parametrize("products", [6, 9])
def test_conv2_fwd_vs_torch(gpu, products):
    """conv2 forward (4x4 stride 2, 20x20x32 -> 9x9x64, bias + ReLU): the
    image-resident kernel (two stages, staging inside the k-steps) with six and
    nine part products vs torch float64:
    max |err| <= 1e-5 * max |ref|.  B = 300 > the persistent grid."""
    Hh = _hip()
    B = 300
    w, packed, pk = _packed(gpu, 64, 21)
    g = torch.Generator().manual_seed(22)
    a1 = torch.relu(torch.randn(B, 20, 20, 32, generator=g))
    b2 = torch.randn(64, generator=g) * 0.1
    a1_d, b2_d = a1.cuda(), b2.cuda()
    out = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
    old = Hh.call("ppo_tune_get", b"products")
    Hh.call("ppo_tune_set", b"products", products)
    try:
        Hh.call("ppo_conv2_fwd", a1_d.data_ptr(), B, pk[0], b2_d.data_ptr(), out.data_ptr(), _s())
        torch.cuda.synchronize()
    finally:
        Hh.call("ppo_tune_set", b"products", old)
    ref = F.conv2d(a1.double().permute(0, 3, 1, 2), w["w2"].double(), b2.double(), stride=2)
    ref = torch.relu(ref).permute(0, 2, 3, 1)
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


def test_conv2_wgrad_vs_torch(gpu):
    """conv2 weight + bias gradient (split-K partials + ppo_wgrad_reduce into the
    torch layout) on the image-resident split-bf16 kernel vs torch float64:
    max |err| <= 1e-5 * max |ref| per tensor.  B = 300."""
    Hh = _hip()
    B = 300
    g = torch.Generator().manual_seed(31)
    a1 = torch.relu(torch.randn(B, 20, 20, 32, generator=g))
    dz2 = torch.randn(B, 9, 9, 64, generator=g)
    a1_d, dz2_d = a1.cuda(), dz2.cuda()
    Z = Hh.call("ppo_wgrad_splits", B * 81, 4, 2048, 16)
    slab = torch.empty(Z * 64 * 512, device=gpu)
    slab_b = torch.empty(Z * 64, device=gpu)
    gw = torch.empty(64 * 512, device=gpu)
    gb = torch.empty(64, device=gpu)
    Hh.call("ppo_conv2_wgrad", dz2_d.data_ptr(), a1_d.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), _s())
    Hh.call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, 64, 512, 1, 4, 32, gw.data_ptr(),
            gb.data_ptr(), 1.0, 0, _s())
    torch.cuda.synchronize()
    x, dy = a1.double().permute(0, 3, 1, 2), dz2.double().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(x, (64, 32, 4, 4), dy, stride=2)
    ref_b = dy.sum((0, 2, 3))
    for got, ref in ((gw.cpu().double().view(64, 32, 4, 4), ref_w), (gb.cpu().double(), ref_b)):
        err = (got - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item(), err


def test_two_rank_update_one_gpu():
    """The N>1 protocol end to end on the device (two processes sharing the one
    GPU, gloo collectives on device tensors; RCCL takes the same calls on an
    8-GPU node): ranks start from different inits, PPO broadcasts rank 0's
    parameters, each rank rolls out its own lanes, the advantage statistics and
    every minibatch gradient are all-reduced -> bit-identical parameters on both
    ranks after the update, and they moved."""
    import json
    import socket
    import subprocess
    import sys
    import os
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    worker = os.path.join(os.path.dirname(__file__), "helpers", "two_rank_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", port], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    for o in outs:
        assert o["same"] and o["moved"] > 1e-6 and all(np.isfinite(o["losses"]))
    assert outs[0]["sum"] == outs[1]["sum"]
    assert outs[0]["losses"] == outs[1]["losses"]


def test_conv3_dgrad_vs_torch(gpu):
    """conv3 dgrad (3x3 stride 1, 7x7x32 -> 9x9x64, a2 ReLU mask) on the
    image-resident split-bf16 kernel vs torch float64:
    max |err| <= 1e-5 * max |ref|.  B = 300 > the persistent grid."""
    Hh = _hip()
    B = 300
    w, packed, pk = _packed(gpu, 64, 41)
    g = torch.Generator().manual_seed(42)
    dz3 = torch.randn(B, 7, 7, 32, generator=g)
    a2 = torch.randn(B, 9, 9, 64, generator=g)
    dz3_d, a2_d = dz3.cuda(), a2.cuda()
    dz2 = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
    Hh.call("ppo_conv3_dgrad", dz3_d.data_ptr(), B, pk[4], a2_d.data_ptr(), dz2.data_ptr(), _s())
    torch.cuda.synchronize()
    ref = F.conv_transpose2d(dz3.double().permute(0, 3, 1, 2), w["w3"].double()).permute(0, 2, 3, 1)
    ref = torch.where(a2 > 0, ref, torch.zeros((), dtype=torch.float64))
    err = (dz2.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


def test_conv3_fwd_vs_torch(gpu):
    """conv3 forward (3x3 stride 1, 9x9x64 -> 7x7x32, bias + ReLU) on the
    image-resident kernel vs torch float64:
    max |err| <= 1e-5 * max |ref|.  B = 300 > the persistent grid."""
    Hh = _hip()
    B = 300
    w, packed, pk = _packed(gpu, 64, 51)
    g = torch.Generator().manual_seed(52)
    a2 = torch.relu(torch.randn(B, 9, 9, 64, generator=g))
    b3 = torch.randn(32, generator=g) * 0.1
    a2_d, b3_d = a2.cuda(), b3.cuda()
    out = torch.full((B, 7, 7, 32), float("nan"), device=gpu)
    Hh.call("ppo_conv3_fwd", a2_d.data_ptr(), B, pk[1], b3_d.data_ptr(), out.data_ptr(), _s())
    torch.cuda.synchronize()
    ref = torch.relu(F.conv2d(a2.double().permute(0, 3, 1, 2), w["w3"].double(), b3.double())).permute(0, 2, 3, 1)
    err = (out.cpu().double() - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item(), err


def test_conv2_fwd_two_stage_bit_identical(gpu):
    """conv2 forward (two compact LDS stages, staging inside the k-steps,
    partials handed over in the vacated stage): the rollout instantiation and
    the training one that also writes the ReLU mask bits give bit-identical
    outputs, and the bits are exactly (out > 0); B = 300 and the rollout-like
    B = 7 (fewer images than blocks)."""
    Hh = _hip()
    _, packed, pk = _packed(gpu, 64, 71)
    g = torch.Generator().manual_seed(72)
    for B in (300, 7):
        a1 = torch.relu(torch.randn(B, 20, 20, 32, generator=g)).cuda()
        b2 = (torch.randn(64, generator=g) * 0.1).cuda()
        o = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
        bits = torch.zeros(B * 81, dtype=torch.int64, device=gpu)
        Hh.call("ppo_conv2_fwd_mask", a1.data_ptr(), B, pk[0], b2.data_ptr(), o.data_ptr(), bits.data_ptr(), _s())
        o2 = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
        Hh.call("ppo_conv2_fwd", a1.data_ptr(), B, pk[0], b2.data_ptr(), o2.data_ptr(), _s())
        torch.cuda.synchronize()
        assert not torch.isnan(o).any()
        assert torch.equal(o, o2)
        pos = (o.reshape(B * 81, 64) > 0).cpu().to(torch.int64)
        want = (pos << torch.arange(64, dtype=torch.int64)).sum(1)
        assert torch.equal(bits.cpu(), want)


def test_stagger_bit_identical(gpu):
    """ppo_tune_set("stagger", 1) only moves waves 4-7's staging of the next image
    behind their compute (conv2 / conv3 dgrad, conv3 forward); bit 2 defers conv2
    dgrad's stores into the next image's k-steps: every output is
    bit-identical to the unstaggered kernels, on B = 300 (> the persistent grid:
    blocks walk several images, both stage parities)."""
    Hh = _hip()
    B = 300
    _, packed, pk = _packed(gpu, 64, 61)
    g = torch.Generator().manual_seed(62)
    dz2 = torch.randn(B, 9, 9, 64, generator=g).cuda()
    dz3 = torch.randn(B, 7, 7, 32, generator=g).cuda()
    a1 = torch.randn(B, 20, 20, 32, generator=g).cuda()
    a2 = torch.relu(torch.randn(B, 9, 9, 64, generator=g)).cuda()
    b3 = (torch.randn(32, generator=g) * 0.1).cuda()

    def run():
        o = [torch.full((B, 20, 20, 32), float("nan"), device=gpu), torch.full((B, 9, 9, 64), float("nan"), device=gpu),
             torch.full((B, 7, 7, 32), float("nan"), device=gpu)]
        Hh.call("ppo_conv2_dgrad", dz2.data_ptr(), B, pk[5], a1.data_ptr(), o[0].data_ptr(), _s())
        Hh.call("ppo_conv3_dgrad", dz3.data_ptr(), B, pk[4], a2.data_ptr(), o[1].data_ptr(), _s())
        Hh.call("ppo_conv3_fwd", a2.data_ptr(), B, pk[1], b3.data_ptr(), o[2].data_ptr(), _s())
        torch.cuda.synchronize()
        return o

    old = Hh.call("ppo_tune_get", b"stagger")
    try:
        Hh.call("ppo_tune_set", b"stagger", 0)
        ref = run()
        got = []
        for v in (1, 2, 3):
            Hh.call("ppo_tune_set", b"stagger", v)
            got.append(run())
    finally:
        Hh.call("ppo_tune_set", b"stagger", old)
    for g_ in got:
        for r, x in zip(ref, g_):
            assert not torch.isnan(r).any()
            assert torch.equal(r, x)


def test_conv3_wgrad_vs_torch(gpu):
    """conv3 weight + bias gradient (partials + ppo_wgrad_reduce into the torch
    layout) on the image-resident split-bf16 kernel vs torch float64:
    max |err| <= 1e-5 * max |ref| per tensor.  B = 300."""
    Hh = _hip()
    B = 300
    g = torch.Generator().manual_seed(61)
    a2 = torch.relu(torch.randn(B, 9, 9, 64, generator=g))
    dz3 = torch.randn(B, 7, 7, 32, generator=g)
    a2_d, dz3_d = a2.cuda(), dz3.cuda()
    Z = Hh.call("ppo_wgrad_splits", B * 49, 5, 2048, 16)
    slab = torch.empty(Z * 32 * 576, device=gpu)
    slab_b = torch.empty(Z * 32, device=gpu)
    gw = torch.empty(32 * 576, device=gpu)
    gb = torch.empty(32, device=gpu)
    Hh.call("ppo_conv3_wgrad", dz3_d.data_ptr(), a2_d.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), _s())
    Hh.call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, 32, 576, 1, 3, 64, gw.data_ptr(),
            gb.data_ptr(), 1.0, 0, _s())
    torch.cuda.synchronize()
    x, dy = a2.double().permute(0, 3, 1, 2), dz3.double().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(x, (32, 64, 3, 3), dy)
    ref_b = dy.sum((0, 2, 3))
    for got, ref in ((gw.cpu().double().view(32, 64, 3, 3), ref_w), (gb.cpu().double(), ref_b)):
        err = (got - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item(), err


def _conv_ops(gpu, B, seed):
    """The six image-resident split kernels on one random problem each; returns
    {name: (gpu fp32 result, float64 reference, torch CPU fp32 result)}."""
    Hh = _hip()
    w, packed, pk = _packed(gpu, 64, seed)
    g = torch.Generator().manual_seed(seed + 1)
    a1 = torch.relu(torch.randn(B, 20, 20, 32, generator=g))
    a2 = torch.relu(torch.randn(B, 9, 9, 64, generator=g))
    dz2 = torch.randn(B, 9, 9, 64, generator=g)
    dz3 = torch.randn(B, 7, 7, 32, generator=g)
    b2, b3 = torch.randn(64, generator=g) * 0.1, torch.randn(32, generator=g) * 0.1
    d = {k: v.cuda() for k, v in dict(a1=a1, a2=a2, dz2=dz2, dz3=dz3, b2=b2, b3=b3).items()}
    s = _s()
    out = {}
    o = torch.empty(B, 9, 9, 64, device=gpu)
    Hh.call("ppo_conv2_fwd", d["a1"].data_ptr(), B, pk[0], d["b2"].data_ptr(), o.data_ptr(), s)
    nchw = lambda t: t.permute(0, 3, 1, 2)
    f = lambda x, w_, b_, st: torch.relu(F.conv2d(nchw(x), w_, b_, stride=st)).permute(0, 2, 3, 1)
    out["conv2_fwd"] = (o, f(a1.double(), w["w2"].double(), b2.double(), 2), f(a1, w["w2"], b2, 2))
    o = torch.empty(B, 7, 7, 32, device=gpu)
    Hh.call("ppo_conv3_fwd", d["a2"].data_ptr(), B, pk[1], d["b3"].data_ptr(), o.data_ptr(), s)
    out["conv3_fwd"] = (o, f(a2.double(), w["w3"].double(), b3.double(), 1), f(a2, w["w3"], b3, 1))
    ct = lambda dz, w_, mask, st: torch.where(mask > 0, F.conv_transpose2d(nchw(dz), w_, stride=st).permute(0, 2, 3, 1),
                                              torch.zeros((), dtype=dz.dtype))
    o = torch.empty(B, 20, 20, 32, device=gpu)
    Hh.call("ppo_conv2_dgrad", d["dz2"].data_ptr(), B, pk[5], d["a1"].data_ptr(), o.data_ptr(), s)
    out["conv2_dgrad"] = (o, ct(dz2.double(), w["w2"].double(), a1, 2), ct(dz2, w["w2"], a1, 2))
    o = torch.empty(B, 9, 9, 64, device=gpu)
    Hh.call("ppo_conv3_dgrad", d["dz3"].data_ptr(), B, pk[4], d["a2"].data_ptr(), o.data_ptr(), s)
    out["conv3_dgrad"] = (o, ct(dz3.double(), w["w3"].double(), a2, 1), ct(dz3, w["w3"], a2, 1))
    for name, x, dz, co, K, ks, st, tap in (("conv2_wgrad", "a1", "dz2", 64, 512, 4, 2, 81),
                                            ("conv3_wgrad", "a2", "dz3", 32, 576, 3, 1, 49)):
        Z = Hh.call("ppo_wgrad_splits", B * tap, 4 if ks == 4 else 5, 2048, 16)
        slab, slab_b = torch.empty(Z * co * K, device=gpu), torch.empty(Z * co, device=gpu)
        gw, gb = torch.empty(co * K, device=gpu), torch.empty(co, device=gpu)
        Hh.call("ppo_" + name, d[dz].data_ptr(), d[x].data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), s)
        Hh.call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, co, K, 1, ks, K // (ks * ks),
                gw.data_ptr(), gb.data_ptr(), 1.0, 0, s)
        xs, dzs = dict(a1=a1, a2=a2)[x], dict(dz2=dz2, dz3=dz3)[dz]
        cw = lambda xx, dd: torch.nn.grad.conv2d_weight(nchw(xx), (co, K // (ks * ks), ks, ks), nchw(dd), stride=st)
        out[name] = (gw.view(co, K // (ks * ks), ks, ks), cw(xs.double(), dzs.double()), cw(xs, dzs))
    torch.cuda.synchronize()
    return out


def test_split_products_fp32_accuracy(gpu):
    """Six part products per operand pair (the default) keep fp32 accuracy: on
    every image-resident split kernel, the error vs float64 (max |err| / max |ref|)
    stays within 2x that of the exact nine-product path and within 4x that of
    torch's own CPU fp32 convolution on the same inputs; both below 1e-6."""
    Hh = _hip()
    B = 300
    res = {}
    for np_ in (9, 6):
        Hh.call("ppo_tune_set", b"products", np_)
        try:
            res[np_] = _conv_ops(gpu, B, 70)
        finally:
            Hh.call("ppo_tune_set", b"products", 6)
    rel = lambda got, ref: ((got.cpu().double() - ref).abs().max() / ref.abs().max()).item()
    for name in res[6]:
        e6 = rel(res[6][name][0], res[6][name][1])
        e9 = rel(res[9][name][0], res[9][name][1])
        ecpu = rel(res[6][name][2], res[6][name][1])
        print(f"{name}: x6 {e6:.3e}  x9 {e9:.3e}  torch-cpu-fp32 {ecpu:.3e}")
        assert e6 <= 2 * e9 + 1e-9 and e6 <= 4 * ecpu + 1e-9 and e6 < 1e-6, (name, e6, e9, ecpu)


@pytest.mark.parametrize("M,H", [(37, 64), (512, 256), (100, 128), (4096, 256), (4001, 512)])
def test_gru_step_kernels_vs_float64(gpu, M, H):
    """The register-tiled GRU step kernels (default) and the tile-GEMM steps
    (ppo_gru_variant_set(1)) vs a float64 restatement of the cell
    (model.py:112-115 with h_in = h·mask): forward outputs, every saved gate, and
    the backward carry (dh_in + dh'·z)·m, within 2e-5 of max|ref|.  M = 4096 / 4000
    (the rollout's rows): the forward step's blocks loop over several row groups
    (at most two blocks per CU), a one-row last group at 4001."""
    Hh = _hip()
    g = torch.Generator().manual_seed(M + H)
    hprev = torch.randn(M, H, generator=g)
    masks = (torch.rand(M, generator=g) > 0.2).float()
    whh = torch.randn(3 * H, H, generator=g) / H ** 0.5
    bhh = torch.randn(3 * H, generator=g) * 0.1
    gi = torch.randn(M, 3 * H, generator=g)
    dgh = torch.randn(M, 3 * H, generator=g)
    dhz = torch.randn(M, H, generator=g)
    d = {k: v.cuda() for k, v in dict(hprev=hprev, masks=masks, whh=whh, bhh=bhh, gi=gi, dgh=dgh, dhz=dhz).items()}
    whhT = d["whh"].t().contiguous()
    hin = hprev.double() * masks.double()[:, None]
    gh = hin @ whh.double().t() + bhh.double()
    gd = gi.double()
    r = torch.sigmoid(gd[:, :H] + gh[:, :H])
    z = torch.sigmoid(gd[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gd[:, 2 * H:] + r * gh[:, 2 * H:])
    ref = {"hout": (1 - z) * n + z * hin, "r": r, "z": z, "n": n, "ghn": gh[:, 2 * H:], "hin": hin,
           "carry": (dgh.double() @ whh.double() + dhz.double()) * masks.double()[:, None]}
    for variant in (0, 1):
        out = {k: torch.full((M, H), float("nan"), device=gpu) for k in ref}
        Hh.call("ppo_gru_variant_set", variant)
        try:
            Hh.call("ppo_gru_step_fwd", d["hprev"].data_ptr(), d["masks"].data_ptr(), None, d["whh"].data_ptr(),
                    d["bhh"].data_ptr(), d["gi"].data_ptr(), M, H, out["hout"].data_ptr(), out["r"].data_ptr(),
                    out["z"].data_ptr(), out["n"].data_ptr(), out["ghn"].data_ptr(), out["hin"].data_ptr(), _s())
            Hh.call("ppo_gru_step_bwd", d["dgh"].data_ptr(), whhT.data_ptr(), d["dhz"].data_ptr(),
                    d["masks"].data_ptr(), None, out["carry"].data_ptr(), M, H, _s())
            torch.cuda.synchronize()
        finally:
            Hh.call("ppo_gru_variant_set", 0)
        for k, v in ref.items():
            err = (out[k].cpu().double() - v).abs().max().item()
            assert err <= 2e-5 * max(v.abs().max().item(), 1.0), (variant, k, err)


@pytest.mark.parametrize("T,n,H,use_idx", [(24, 512, 256, True), (9, 37, 64, False), (5, 100, 128, True),
                                            (3, 16, 512, False)])
def test_gru_persistent_sequence_equals_steps(gpu, T, n, H, use_idx):
    """ppo_gru_seq_fwd as one persistent launch (row groups synchronised by
    release/acquire counters, W_hh slices resident) equals the step-by-step
    launches bit for bit — hout and every saved gate over all T steps — with masks
    direct ([T][n]) or through the minibatch index, and no bounded wait timed out."""
    Hh = _hip()
    g = torch.Generator().manual_seed(T * n + H)
    N = 3 * n
    h0 = torch.randn(n, H, generator=g).cuda()
    whh = (torch.randn(3 * H, H, generator=g) / H ** 0.5).cuda()
    bhh = (torch.randn(3 * H, generator=g) * 0.1).cuda()
    gi = torch.randn(T * n, 3 * H, generator=g).cuda()
    if use_idx:
        masks = (torch.rand(T * N, generator=g) > 0.1).float().cuda()
        idx = torch.randint(0, T * N, (T * n,), generator=g).cuda()
    else:
        masks = (torch.rand(T * n, generator=g) > 0.1).float().cuda()
        idx = None
    outs = {}
    prev = Hh.call("ppo_gru_persist_get")
    for persist in (0, 1):   # step launches, persistent launch
        o = {k: torch.full((T * n, H), float("nan"), device=gpu) for k in ("h", "r", "z", "n", "ghn", "hin")}
        Hh.call("ppo_gru_persist_set", persist)
        try:
            Hh.call("ppo_gru_seq_fwd", h0.data_ptr(), masks.data_ptr(), None if idx is None else idx.data_ptr(),
                    whh.data_ptr(), bhh.data_ptr(), gi.data_ptr(), T, n, H, o["h"].data_ptr(), o["r"].data_ptr(),
                    o["z"].data_ptr(), o["n"].data_ptr(), o["ghn"].data_ptr(), o["hin"].data_ptr(), _s())
            torch.cuda.synchronize()
        finally:
            Hh.call("ppo_gru_persist_set", prev)
        outs[persist] = o
        assert Hh.call("ppo_gru_persist_timeouts", _s()) == 0, persist
    for p in (1,):
        for k in outs[0]:
            assert torch.isfinite(outs[p][k]).all(), (p, k)
            assert torch.equal(outs[0][k], outs[p][k]), (p, k, (outs[0][k] - outs[p][k]).abs().max().item(),
                                                          (outs[0][k] != outs[p][k]).sum().item())


@pytest.mark.parametrize("T,n,H,use_idx", [(24, 512, 256, True), (9, 37, 64, False), (5, 100, 128, True),
                                            (3, 16, 512, False), (2, 64, 256, True), (256, 512, 256, True),
                                            (48, 512, 64, True), (40, 256, 64, False)])
def test_gru_persistent_bptt_equals_steps(gpu, T, n, H, use_idx):
    """ppo_gru_seq_bwd_ws as one persistent launch (gru_seq_bwd16_kernel: W_hh^T
    slices resident, dgh handed over between the unit blocks of a row group by sc1
    stores and loads) equals the T - 1 step launches bit for bit — dgi and dgh over
    all T steps, the final dhz and carry — with masks direct or through the minibatch
    index, and the error word stays clear; every group reports that it ran the
    persistent kernel — at c5's shape (T = 256, n = 512, H = 256) among others."""
    Hh = _hip()
    g = torch.Generator().manual_seed(T * n + H + 1)
    N = 3 * n
    R = T * n
    G = (n + 31) // 32
    dout = torch.randn(R, H, generator=g).cuda()
    sv = {"r": torch.rand(R, H, generator=g), "z": torch.rand(R, H, generator=g),
          "n": torch.rand(R, H, generator=g) * 2 - 1, "ghn": torch.randn(R, H, generator=g),
          "hin": torch.randn(R, H, generator=g)}
    sv = {k: v.cuda() for k, v in sv.items()}
    whhT = (torch.randn(H, 3 * H, generator=g) / H ** 0.5).cuda()
    if use_idx:
        masks = (torch.rand(T * N, generator=g) > 0.1).float().cuda()
        idx = torch.randint(0, T * N, (R,), generator=g).cuda()
    else:
        masks = (torch.rand(R, generator=g) > 0.1).float().cuda()
        idx = None
    cnt = torch.zeros(Hh.call("ppo_gru_seq_counters", n), dtype=torch.int32, device=gpu)
    assert cnt.numel() == 2 * G
    err = torch.zeros(1, dtype=torch.int32, device=gpu)
    outs = {}
    prev = Hh.call("ppo_gru_persist_get")
    paths = None
    for persist in (0, 3):
        o = {"dgi": torch.full((R, 3 * H), float("nan"), device=gpu), "dgh": torch.full((R, 3 * H), float("nan"),
                                                                                       device=gpu),
             "dhz": torch.zeros(n, H, device=gpu), "carry": torch.zeros(n, H, device=gpu)}
        Hh.call("ppo_gru_persist_set", persist)
        try:
            Hh.call("ppo_gru_seq_bwd_ws", dout.data_ptr(), sv["r"].data_ptr(), sv["z"].data_ptr(), sv["n"].data_ptr(),
                    sv["ghn"].data_ptr(), sv["hin"].data_ptr(), masks.data_ptr(),
                    None if idx is None else idx.data_ptr(), whhT.data_ptr(), T, n, H, o["dgi"].data_ptr(),
                    o["dgh"].data_ptr(), o["dhz"].data_ptr(), o["carry"].data_ptr(), cnt.data_ptr(), err.data_ptr(),
                    _s())
            torch.cuda.synchronize()
        finally:
            Hh.call("ppo_gru_persist_set", prev)
        outs[persist] = o
        if persist == 3 and T > 1 and G * (H // 16) <= torch.cuda.get_device_properties(0).multi_processor_count:
            paths = cnt[G:].cpu()
    assert err.item() == 0
    if paths is not None:
        assert (paths == 1).all(), paths
    outs[1] = outs.pop(3)
    for k in outs[0]:
        assert torch.isfinite(outs[1][k]).all(), k
        bad = (outs[0][k] != outs[1][k]).nonzero()
        if bad.numel():
            rows = bad[:, 0].cpu()
            print(k, "mismatches", bad.shape[0], "steps", torch.unique(rows // n).tolist()[:20],
                  "cols", torch.unique(bad[:, 1].cpu() % H).tolist()[:20], "gate", torch.unique(bad[:, 1].cpu() // H).tolist())
        assert torch.equal(outs[0][k], outs[1][k]), (k, (outs[0][k] - outs[1][k]).abs().max().item())


def test_gru_persistent_bptt_timeout_sets_error(gpu):
    """a bounded wait of the persistent BPTT that runs out (spin bound 0) sets the
    error word and the launch returns; a launch that starts with the word set
    returns at once (outputs untouched), and with the default bound it completes."""
    Hh = _hip()
    T, n, H = 6, 256, 256
    g = torch.Generator().manual_seed(9)
    R = T * n
    args = [torch.randn(R, H, generator=g).cuda() for _ in range(6)]
    masks = torch.ones(R, device=gpu)
    whhT = (torch.randn(H, 3 * H, generator=g) / 16).cuda()
    dgi = torch.zeros(R, 3 * H, device=gpu)
    dgh = torch.zeros(R, 3 * H, device=gpu)
    dhz = torch.zeros(n, H, device=gpu)
    carry = torch.zeros(n, H, device=gpu)
    cnt = torch.zeros(Hh.call("ppo_gru_seq_counters", n), dtype=torch.int32, device=gpu)
    err = torch.zeros(1, dtype=torch.int32, device=gpu)

    def run():
        Hh.call("ppo_gru_seq_bwd_ws", *[a.data_ptr() for a in args], masks.data_ptr(), None, whhT.data_ptr(), T, n,
                H, dgi.data_ptr(), dgh.data_ptr(), dhz.data_ptr(), carry.data_ptr(), cnt.data_ptr(), err.data_ptr(),
                _s())
        torch.cuda.synchronize()
    prev = Hh.call("ppo_gru_persist_get")
    Hh.call("ppo_gru_persist_set", 3)
    Hh.call("ppo_gru_persist_spin_set", 0)
    try:
        run()
    finally:
        Hh.call("ppo_gru_persist_spin_set", 1 << 21)
    assert err.item() == 1
    dgi.zero_()
    run()                       # sticky: returns at once
    assert err.item() == 1
    assert (dgi[: (T - 1) * n] == 0).all()
    err.zero_()
    try:
        run()
    finally:
        Hh.call("ppo_gru_persist_set", prev)
    assert err.item() == 0 and torch.isfinite(dgi).all() and (dgi[: n] != 0).any()


@pytest.mark.parametrize("variant,Z", [(5, 0), (8, 0), (8, 256), (9, 0), (9, 256), (9, 7), (10, 0), (10, 256), (10, 7)])
def test_conv1_wgrad_variants_vs_torch(gpu, variant, Z):
    """conv1 weight + bias gradient from u8 observations gathered by index (the
    minibatch path): the part-pipelined bf16x3 kernel (5, 16 waves, two tiles per
    wave), the k-split kernels of conv1w.hip (8; 9 and 10 with one / two waves per SIMD; Z =
    256 leaves blocks with one and two of the B = 300 images, Z = 7 walks 42-43
    images per block) vs torch float64 on (u8 / 255):
    max |err| <= 1e-5 * max |ref|.  Rows gathered out of order."""
    Hh = _hip()
    B, rows = 300, 420
    g = torch.Generator().manual_seed(81)
    obs = torch.randint(0, 256, (rows, 4, 84, 84), dtype=torch.uint8, generator=g)
    idx = torch.randperm(rows, generator=g)[:B].contiguous()
    dz1 = torch.randn(B, 20, 20, 32, generator=g)
    obs_d, idx_d, dz1_d = obs.cuda(), idx.cuda(), dz1.cuda()
    Z = Z or Hh.call("ppo_wgrad_splits", B * 400, 1, 2048, 16)
    slab = torch.empty(Z * 32 * 256, device=gpu)
    slab_b = torch.empty(Z * 32, device=gpu)
    gw = torch.empty(32 * 256, device=gpu)
    gb = torch.empty(32, device=gpu)
    old = Hh.call("ppo_tune_get", b"conv1_wgrad")
    Hh.call("ppo_tune_set", b"conv1_wgrad", variant)
    try:
        Hh.call("ppo_conv1_wgrad", dz1_d.data_ptr(), obs_d.data_ptr(), 1, idx_d.data_ptr(), 0, 4, B, Z,
                slab.data_ptr(), slab_b.data_ptr(), _s())
        Hh.call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, 32, 256, 0, 0, 0, gw.data_ptr(),
                gb.data_ptr(), 1.0 / 255, 0, _s())
        torch.cuda.synchronize()
    finally:
        Hh.call("ppo_tune_set", b"conv1_wgrad", old)
    x = obs[idx].double() / 255.0
    dy = dz1.double().permute(0, 3, 1, 2)
    ref_w = torch.nn.grad.conv2d_weight(x, (32, 4, 8, 8), dy, stride=4)
    ref_b = dy.sum((0, 2, 3))
    for got, ref in ((gw.cpu().double().view(32, 4, 8, 8), ref_w), (gb.cpu().double(), ref_b)):
        err = (got - ref).abs().max().item()
        assert err <= 1e-5 * ref.abs().max().item(), err


def _run_procs(cmds, timeout=300):
    import subprocess
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for c in cmds]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-3000:]
        outs.append(o)
    return outs


def test_split_minibatch_gradient_equals_single_gpu(tmp_path):
    """the same global minibatch on one rank, or split over two
    ranks that each own half of the env lanes (gloo on the one GPU; RCCL takes the
    same calls on a node), gives the same averaged gradient — global advantage
    statistics from the 3-double all-reduce, per-rank mean over B/2 rows, Σ/G of
    the all-reduced flat gradient.  Tolerance: 2e-6 of each tensor's max |g|
    (only the fp32 summation order differs), losses 1e-6 relative."""
    import os
    import socket
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    worker = os.path.join(os.path.dirname(__file__), "helpers", "split_grad_worker.py")
    one, two = str(tmp_path / "g1.npz"), str(tmp_path / "g2.npz")
    _run_procs([[sys.executable, worker, "0", "1", port, one]])
    _run_procs([[sys.executable, worker, str(r), "2", port, two] for r in range(2)])
    a, b = np.load(one), np.load(two)
    np.testing.assert_allclose(b["stats"], a["stats"], rtol=1e-12)
    np.testing.assert_allclose(b["loss"][:3], a["loss"][:3], rtol=1e-6, atol=1e-9)
    shapes = O.cnn_param_shapes(128)
    ga, gb = O.unflatten(a["grad"], shapes), O.unflatten(b["grad"], shapes)
    for name, _ in shapes:
        ref = ga[name]
        err = np.abs(gb[name] - ref).max()
        assert err <= 2e-6 * max(np.abs(ref).max(), 1e-6), (name, err, np.abs(ref).max())


def test_bench_self_launches_ranks():
    """`bench.py --gpus 2` without a launcher starts its two ranks itself (here
    both on the one GPU with --dist-backend gloo) and reports n_gpus 2; a
    WORLD_SIZE that disagrees with --gpus is refused."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "1",
           "--warmup", "0", "--envs", "64", "--num-steps", "8", "--no-cpu-baseline", "--no-gae-roofline",
           "--no-boundary", "--no-profile-pass"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["config"]["global_batch"] == 2 * 64 * 8 and line["value"] > 0
    bad = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(cmd, env=bad, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "does not match" in r.stderr


@pytest.mark.parametrize("use_gae", [True, False])
@pytest.mark.parametrize("ptl", [True, False])
@pytest.mark.parametrize("T,N", [(128, 8), (128, 1024), (77, 1031), (5, 1), (300, 33), (1, 17)])
def test_gae_time_parallel_scan(gpu, use_gae, ptl, T, N):
    """ppo_compute_returns_scan (time-parallel affine scan, storage.py:82-121 in
    every branch) vs the C oracle (the reference's fp32 op order): returns within
    2e-6 of max|returns| (reassociation only), the storage side effect on
    value_preds[T] / returns[T] exact, fused advantages + moments vs the oracle."""
    H = _hip()
    rng = np.random.default_rng(T * 31 + N + 7 * use_gae + ptl)
    r = rng.random((T, N), np.float32)
    v = (3 * rng.standard_normal((T + 1, N))).astype(np.float32)
    m = (rng.random((T + 1, N)) > 0.05).astype(np.float32)
    bm = (rng.random((T + 1, N)) > 0.05).astype(np.float32)
    nv = rng.standard_normal(N).astype(np.float32)
    rd, vd, md, bmd, nvd = _dev(r), _dev(v), _dev(m), _dev(bm), _dev(nv)
    ret = torch.zeros(T + 1, N, device=gpu)
    adv = torch.zeros(T, N, device=gpu)
    nparts = H.call("ppo_gae_scan_partials_count", N)
    parts = torch.zeros(3 * nparts, dtype=torch.float64, device=gpu)
    stats = torch.zeros(3, dtype=torch.float64, device=gpu)
    H.call("ppo_compute_returns_scan", rd.data_ptr(), vd.data_ptr(), md.data_ptr(), bmd.data_ptr(), nvd.data_ptr(),
           ret.data_ptr(), adv.data_ptr(), parts.data_ptr(), T, N, 0.99, 0.95, int(use_gae), int(ptl), _s())
    H.call("ppo_adv_finalize", parts.data_ptr(), nparts, float(T * N), stats.data_ptr(), _s())
    eret, ev = O.compute_returns(r, v, m, bm, nv, use_gae, 0.99, 0.95, ptl)
    got = ret.cpu().numpy()
    scale = np.abs(eret[:T]).max()
    np.testing.assert_allclose(got[:T], eret[:T], rtol=0, atol=2e-6 * scale)
    assert np.array_equal(vd.cpu().numpy(), ev)               # value_preds[T] = next_value (GAE)
    if not use_gae:
        assert np.array_equal(got[T], nv)                     # returns[T] = next_value
    d = got[:T].astype(np.float64) - v[:T]
    np.testing.assert_allclose(adv.cpu().numpy(), d, rtol=0, atol=2e-6 * scale)
    st = stats.cpu().numpy()   # {count, mean, M2} (Welford / Chan)
    assert st[0] == d.size
    np.testing.assert_allclose(st[1], d.mean(), rtol=1e-6, atol=1e-6 * scale)
    np.testing.assert_allclose(st[2], ((d - d.mean()) ** 2).sum(), rtol=1e-5)


def test_storage_gae_mode_scan(gpu):
    """RolloutStorage(gae_mode="scan") drives the time-parallel kernel through the
    drop-in API at c2's shape: returns and normalised advantages within
    tolerance of the bit-exact default."""
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    T, N = 128, 1024
    g = torch.Generator().manual_seed(3)
    outs = []
    for mode in ("exact", "scan"):
        st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), 1, obs_dtype=torch.uint8, device=gpu, gae_mode=mode)
        g.manual_seed(3)
        st.rewards.copy_(torch.rand(T, N, 1, generator=g))
        st.value_preds.copy_(torch.randn(T + 1, N, 1, generator=g))
        st.masks.copy_((torch.rand(T + 1, N, 1, generator=g) > 0.01).float())
        st.compute_returns(torch.randn(N, 1, generator=g).to(gpu), True, 0.99, 0.95, False)
        outs.append((st.returns.cpu().numpy(), st.normalized_advantages().cpu().numpy()))
    scale = np.abs(outs[0][0]).max()
    np.testing.assert_allclose(outs[1][0], outs[0][0], rtol=0, atol=2e-6 * scale)
    np.testing.assert_allclose(outs[1][1], outs[0][1], rtol=0, atol=1e-5)
    with pytest.raises(ValueError):
        RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), 1, device=gpu, gae_mode="fast")
