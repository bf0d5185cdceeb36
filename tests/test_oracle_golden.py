"""The oracle (oracle/) pinned against vectors recorded from the reference itself
(tools/gen_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import golden
from oracle import ppo_oracle as O


@pytest.mark.parametrize("gi", [0, 1])
@pytest.mark.parametrize("use_gae", [True, False])
@pytest.mark.parametrize("ptl", [True, False])
def test_gae_bit_exact(gi, use_gae, ptl):
    d = golden("gae.npz")
    k = f"g{gi}_gae{int(use_gae)}_ptl{int(ptl)}"
    ret0 = np.full(d["value_preds"].shape[:2], -7.0, np.float32)
    args = (d["rewards"][..., 0], d["value_preds"][..., 0], d["masks"][..., 0], d["bad_masks"][..., 0],
            d["next_value"][:, 0], use_gae, d["gammas"][gi], d["lambdas"][gi], ptl)
    for fn in (O.compute_returns, O.compute_returns_np):
        ret, v = fn(*args, returns=ret0)
        assert np.array_equal(ret, d[k + "_returns"][..., 0])          # bit-exact
        assert np.array_equal(v, d[k + "_value_preds"][..., 0])


@pytest.mark.parametrize("c", [0, 1, 2])
def test_advantage_normalisation(c):
    d = golden("advnorm.npz")
    a = O.normalize_advantages(d[f"c{c}_returns"][..., 0], d[f"c{c}_value_preds"][..., 0])
    np.testing.assert_allclose(a, d[f"c{c}_advantages"][..., 0], rtol=1e-6, atol=1e-6)


def test_sampler_cuts():
    import torch
    d = golden("sampler.npz")
    for c in range(4):
        seed, T, N, M = d[f"c{c}_meta"]
        torch.manual_seed(int(seed))
        perm = torch.randperm(int(T * N)).numpy()
        got = np.stack(O.ff_minibatches(perm, int(M)))
        assert np.array_equal(got, d[f"c{c}_ff"])
        if f"c{c}_rec" in d:
            torch.manual_seed(int(seed))
            perm = torch.randperm(int(N)).numpy()
            envs = O.rec_minibatches(perm, int(M))
            rows = np.stack([(np.arange(T)[:, None] * N + e[None, :]).reshape(-1) for e in envs])
            assert np.array_equal(rows, d[f"c{c}_rec"])


def test_recurrent_sampler_ragged_raises():
    with pytest.raises(IndexError):
        O.rec_minibatches(np.arange(7), 3)


def test_categorical():
    d = golden("categorical.npz")
    c = O.categorical(d["logits_raw"], d["exp_noise"])
    assert np.array_equal(c["action"], d["action"][:, 0])
    assert np.array_equal(O.categorical(d["logits_raw"])["action"], d["mode"][:, 0])
    np.testing.assert_allclose(c["log_prob"], d["log_probs"][:, 0], rtol=0, atol=2e-6)
    np.testing.assert_allclose(c["entropy"], d["entropy"], rtol=0, atol=2e-6)
    np.testing.assert_allclose(c["norm_logits"], d["norm_logits"], rtol=0, atol=2e-6)


def test_adam_clip():
    d = golden("adam_clip.npz")
    p = d["init"].astype(np.float64)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    for k in range(d["grads"].shape[0]):
        p, m, v, gc, tn = O.clip_adam(p, d["grads"][k].astype(np.float64), m, v, k + 1,
                                      float(d["lr"][0]), float(d["eps"][0]), float(d["max_norm"][0]))
        np.testing.assert_allclose(tn, d["total_norms"][k], rtol=1e-6)
        np.testing.assert_allclose(gc, d["clipped"][k], rtol=1e-5, atol=1e-9)
        np.testing.assert_allclose(p, d["after"][k], rtol=0, atol=2e-7)


def test_mlp_submodules():
    """oracle.mlp_forward against MLPBase's submodules (actor / critic /
    critic_linear) and Categorical driven by the reference (mlp.npz)."""
    d = golden("mlp.npz")
    sh = O.mlp_param_shapes(4, 64, 2)
    assert ["base." + str(n) for n in d["base_names"]] == [n for n, _ in sh[:10]]
    p = O.unflatten(np.concatenate([d["base_params"], d["head_params"]]), sh)
    value, logits, cache = O.mlp_forward(p, d["x"])
    np.testing.assert_allclose(value, d["value"][:, 0], atol=1e-6)
    np.testing.assert_allclose(cache["actor"][1], d["actor_features"], atol=1e-6)
    c = O.categorical(logits)
    np.testing.assert_allclose(c["norm_logits"], d["norm_logits"], atol=1e-6)
    np.testing.assert_allclose(c["entropy"], d["entropy"], atol=1e-6)


def test_mlp_backward_finite_difference():
    """oracle.mlp_backward (tanh towers) against central differences of the
    PPO loss in float64."""
    rng = np.random.default_rng(3)
    sh = O.mlp_param_shapes(6, 8, 3)
    p = {n: rng.standard_normal(s) * 0.5 for n, s in sh}
    B = 5
    x = rng.standard_normal((B, 6))
    act = rng.integers(0, 3, B)
    olp, adv = np.log(rng.random(B)) * 0.3 - 1.0, rng.standard_normal(B)
    vp, ret = rng.standard_normal(B) * 0.1, rng.standard_normal(B)

    def loss(q):
        v, lg, _ = O.mlp_forward(q, x)
        r = O.loss_head_grads(v, lg, act, olp, adv, vp, ret, 0.2, 0.5, 0.01)
        return 0.5 * r["value_loss"] + r["action_loss"] - 0.01 * r["entropy"]

    v, lg, cache = O.mlp_forward(p, x)
    r = O.loss_head_grads(v, lg, act, olp, adv, vp, ret, 0.2, 0.5, 0.01)
    g = O.mlp_backward(p, cache, r["g_value"], r["g_logits"])
    for name, shp in sh:
        for j in rng.choice(int(np.prod(shp)), size=min(3, int(np.prod(shp))), replace=False):
            q = {k: a.copy() for k, a in p.items()}
            q[name].reshape(-1)[j] += 1e-6
            lp = loss(q)
            q[name].reshape(-1)[j] -= 2e-6
            lm = loss(q)
            fd = (lp - lm) / 2e-6
            assert abs(fd - g[name].reshape(-1)[j]) < 1e-6 + 1e-5 * abs(fd), (name, j, fd, g[name].reshape(-1)[j])


def test_cartpole_restatement_terminates_and_resets():
    """oracle.cartpole_step: always pushing right topples the pole within gym's
    thresholds; ended lanes report their length and restart in U(-0.05, 0.05)."""
    N = 16
    st, k, obs, *_ = O.cartpole_step(np.zeros((N, 4)), np.zeros(N), None, 7, 0)
    assert np.all(np.abs(obs) <= 0.05) and np.all(k == 0)
    lens = []
    for c in range(1, 200):
        st, k, obs, rew, mask, bad, ep = O.cartpole_step(st, k, np.ones(N, np.int64), 7, c)
        assert np.all(rew == 1) and np.all(bad == 1)
        lens += list(ep[mask == 0])
        assert np.all(np.abs(obs[mask == 0]) <= 0.05)
    assert len(lens) >= N and 5 <= min(lens) and max(lens) <= 30
    st, k, *_ = O.cartpole_step(np.zeros((2, 4)), np.array([0, 9]), np.array([0, 1]), 7, 0, max_steps=10)
    assert list(k) == [1, 0]


def test_torch_ref_replays_reference_iteration():
    """oracle/torch_ref.py (the reference's CPU path restated in torch: the CPU
    baseline bench.py times, and the float64 gradient of tests/test_full_size.py)
    replays the recorded reference iteration: same actions (bit-exact), returns,
    losses and final parameters."""
    import torch
    from oracle import torch_ref as TR
    d = golden("cnn_update.npz")
    hidden, N, T, E, Mb = (int(x) for x in d["meta"])
    torch.set_num_threads(1)
    p = TR.unflatten(torch.from_numpy(d["init_params"]), hidden, requires_grad=True)
    obs = torch.from_numpy(d["obs_u8"]).float() / 255.0
    noise = torch.from_numpy(d["exp_noise"])
    vpred = torch.zeros(T + 1, N, 1)
    logps = torch.zeros(T, N, 1)
    actions = torch.zeros(T, N, 1, dtype=torch.int64)
    masks = torch.ones(T + 1, N, 1)
    masks[1:] = torch.from_numpy(d["masks"])
    for t in range(T):
        with torch.no_grad():
            v, a, lp = TR.act(p, obs[t], noise=noise[t])
        vpred[t], actions[t], logps[t] = v, a, lp
    assert np.array_equal(actions.numpy(), d["actions"])
    np.testing.assert_allclose(logps.numpy(), d["action_log_probs"], atol=1e-6)
    with torch.no_grad():
        nv, _ = TR.cnn_forward(p, obs[-1])
    ret = TR.compute_returns(torch.from_numpy(d["rewards"]), vpred, masks, nv, 0.99, 0.95)
    np.testing.assert_allclose(ret.numpy(), d["returns"], atol=1e-6)
    opt = torch.optim.Adam(p, lr=float(d["lr"][0]), eps=1e-5)
    losses = TR.ppo_update(p, opt, obs, actions, logps, vpred, ret, ppo_epoch=E, num_mini_batch=Mb, clip=0.1,
                           value_coef=0.5, entropy_coef=0.001, max_grad_norm=0.5, perms=torch.from_numpy(d["perms"]))
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-5, atol=1e-7)
    final = torch.cat([t.detach().reshape(-1) for t in p]).numpy()
    np.testing.assert_allclose(final, d["final_params"], rtol=0, atol=1e-6)


def test_torch_ref_minibatch_grads_match_oracle():
    """torch_ref.minibatch_grads (chunked float64 autograd) equals the oracle's
    analytic float64 backward on the same minibatch (independent derivations)."""
    import torch
    from oracle import torch_ref as TR
    rng = np.random.default_rng(8)
    H, B = 64, 12
    shapes = O.cnn_param_shapes(H)
    flat = np.concatenate([rng.standard_normal(int(np.prod(s))) * 0.05 for _, s in shapes])
    obs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
    act = rng.integers(0, 8, B)
    olp, adv = np.log(rng.random(B)) * 0.3 - 2.0, rng.standard_normal(B)
    vp, ret = rng.standard_normal(B) * 0.1, rng.standard_normal(B)
    p = TR.unflatten(torch.from_numpy(flat), H, dtype=torch.float64, requires_grad=True)
    t = lambda a: torch.from_numpy(np.asarray(a))  # noqa: E731
    grads, losses = TR.minibatch_grads(p, t(obs), t(act), t(olp), t(adv), t(vp), t(ret), clip=0.1, value_coef=0.5,
                                       entropy_coef=0.01, chunk=5)
    po = O.unflatten(flat, shapes)
    value, logits, cache = O.cnn_forward(po, obs.astype(np.float64) / 255.0)
    lg = O.loss_head_grads(value, logits, act, olp, adv, vp, ret, 0.1, 0.5, 0.01)
    ref = O.cnn_backward(po, cache, lg["g_value"], lg["g_logits"])
    for (name, _), g in zip(shapes, grads):
        np.testing.assert_allclose(g.numpy(), ref[name], rtol=1e-9, atol=1e-12 * max(1.0, np.abs(ref[name]).max()))
    np.testing.assert_allclose(losses, [lg["value_loss"], lg["action_loss"], lg["entropy"]], rtol=1e-10)


def _gru_step_forward(p, obs_u8, vec, h, mask):
    """The act path of a recurrent CNNBase (model.py:111-115 single-step branch)."""
    feat, _ = O.cnn_trunk(p, O.decode_obs(obs_u8))
    x = np.concatenate([feat, np.asarray(vec, np.float64)], 1)
    h = O.gru_cell(p, x, np.asarray(h, np.float64) * np.asarray(mask, np.float64).reshape(-1, 1))
    value, logits = O.heads(p, h)
    return value, logits, h


def test_oracle_replays_reference_recurrent_rollout():
    """gru_update.npz (tools/gen_golden.py gen_gru_update: the reference's own
    T/ GRU + vector-obs Policy): the oracle's single-step forward replays the
    rollout — actions bit-exact from the recorded Exp(1) noise, values and
    log-probs within 1e-6, the carried hidden state within 1e-6."""
    d = golden("gru_update.npz")
    hidden, V, N, T, E, Mb = (int(x) for x in d["meta"])
    shapes = O.cnn_param_shapes(hidden, recurrent=True, vector_obs_len=V)
    assert [str(n) for n in d["names"]] == [n for n, _ in shapes]
    p = O.unflatten(d["init_params"], shapes)
    h = d["h0"].astype(np.float64)
    masks = np.concatenate([d["masks0"][None], d["masks"]], 0)[..., 0]
    for t in range(T):
        value, logits, h = _gru_step_forward(p, d["obs_u8"][t], d["vector_obs"][t], h, masks[t])
        c = O.categorical(logits, d["exp_noise"][t])
        assert np.array_equal(c["action"], d["actions"][t][:, 0]), t
        np.testing.assert_allclose(value, d["values"][t][:, 0], atol=1e-6)
        np.testing.assert_allclose(c["log_prob"], d["action_log_probs"][t][:, 0], atol=1e-6)
    np.testing.assert_allclose(h, d["hidden_T"], atol=1e-6)
    nv, _, _ = _gru_step_forward(p, d["obs_u8"][T], d["vector_obs"][T], h, masks[T])
    np.testing.assert_allclose(nv, d["next_value"][:, 0], atol=1e-6)


def test_oracle_recurrent_update_pinned_to_reference():
    """The recurrent PPO.update recorded from the reference (recurrent_generator
    env orders, GRU BPTT over masked sequences, clip_grad_norm_, Adam; E = 2,
    M = 2): oracle.run_update_recurrent's first-minibatch gradient (BPTT included)
    equals the reference's within 1e-5 of each tensor's max |g|, every
    minibatch's (value loss, action loss, entropy) and total norm within 1e-5
    relative, the last minibatch's gradient within 1e-3 of max |g| (three fp32 vs
    float64 Adam steps in between move ReLU boundaries of the conv trunk: 2e-4
    measured on conv2), the final parameters within 2e-5 (4e-7 measured)."""
    d = golden("gru_update.npz")
    hidden, V, N, T, E, Mb = (int(x) for x in d["meta"])
    clip, vcoef, ecoef = (float(x) for x in d["coefs"])
    shapes = O.cnn_param_shapes(hidden, recurrent=True, vector_obs_len=V)
    masks = np.concatenate([d["masks0"][None], d["masks"]], 0)[..., 0]
    r = O.run_update_recurrent(d["init_params"], shapes, d["obs_u8"], d["vector_obs"], d["h0"], masks,
                               d["actions"][..., 0], d["action_log_probs"][..., 0], d["value_preds_after"][..., 0],
                               d["returns"][..., 0], d["perms"], num_mini_batch=Mb, clip=clip, value_coef=vcoef,
                               entropy_coef=ecoef, lr=float(d["lr"][0]))
    for got, ref, tol in ((r["preclip_grads"][0], d["mb0_preclip_grad"], 1e-5),
                          (r["preclip_grads"][-1], d["last_preclip_grad"], 1e-3)):
        g, rf = O.unflatten(got, shapes), O.unflatten(ref, shapes)
        for name, _ in shapes:
            err = np.abs(g[name] - rf[name]).max()
            assert err <= tol * max(np.abs(rf[name]).max(), 1e-6), (name, err, np.abs(rf[name]).max())
    np.testing.assert_allclose(r["mb_losses"], d["mb_losses"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(r["total_norms"], d["total_norms"], rtol=1e-5)
    np.testing.assert_allclose(r["losses"], d["losses"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(r["final_params"], d["final_params"], rtol=0, atol=2e-5)


def test_oracle_gru_backward_vs_finite_difference():
    """oracle.gru_backward (the BPTT the GPU kernels are checked against) vs
    central finite differences of gru_sequence_cache in float64, masks with zeros
    included: every weight / bias gradient and dx within 1e-6 relative."""
    rng = np.random.default_rng(17)
    T, n, I, H = 5, 3, 6, 4
    p = {"base.gru.weight_ih_l0": rng.standard_normal((3 * H, I)) * 0.5,
         "base.gru.weight_hh_l0": rng.standard_normal((3 * H, H)) * 0.5,
         "base.gru.bias_ih_l0": rng.standard_normal(3 * H) * 0.3,
         "base.gru.bias_hh_l0": rng.standard_normal(3 * H) * 0.3}
    x = rng.standard_normal((T * n, I))
    h0 = rng.standard_normal((n, H))
    masks = (rng.random((T, n)) > 0.3).astype(np.float64)
    w = rng.standard_normal((T * n, H))     # loss = sum(w * outputs)

    def loss(pp, xx):
        out, _ = O.gru_sequence_cache(pp, xx, h0, masks)
        return float((w * out).sum())

    _, cache = O.gru_sequence_cache(p, x, h0, masks)
    g, dx = O.gru_backward(p, x, masks, cache, w)
    eps = 1e-6
    for k in p:
        fd = np.zeros_like(p[k])
        for i in np.ndindex(p[k].shape):
            q = {kk: vv.copy() for kk, vv in p.items()}
            q[k][i] += eps
            lp = loss(q, x)
            q[k][i] -= 2 * eps
            fd[i] = (lp - loss(q, x)) / (2 * eps)
        np.testing.assert_allclose(g[k], fd, rtol=1e-6, atol=1e-8, err_msg=k)
    fdx = np.zeros_like(x)
    for i in np.ndindex(x.shape):
        xx = x.copy()
        xx[i] += eps
        lp = loss(p, xx)
        xx[i] -= 2 * eps
        fdx[i] = (lp - loss(p, xx)) / (2 * eps)
    np.testing.assert_allclose(dx, fdx, rtol=1e-6, atol=1e-8)


# --------------------------------------------- production hidden sizes
def _digest_check(got_flat, d, prefix, shapes, tol, rel=True, scale=1.0):
    """A fixture digest (tools/gen_golden.py digest: every 8th element, per-tensor
    max |x| and L2) against a full flat array.  rel: sampled elements within tol x
    the tensor's max |x| and each tensor's L2 within 1e-5 relative (gradients); else
    within tol absolute and the L2 within tol x sqrt(numel) (parameters)."""
    idx = d[f"{prefix}_idx"]
    ref = d[f"{prefix}_sampled"].astype(np.float64) * scale
    got = np.asarray(got_flat, np.float64)
    off = 0
    for k, (name, shape) in enumerate(shapes):
        n = int(np.prod(shape))
        sel = (idx >= off) & (idx < off + n)
        tmax = d[f"{prefix}_tmax"][k] * scale
        err = np.abs(got[idx[sel]] - ref[sel]).max()
        l2, l2ref = np.sqrt((got[off:off + n] ** 2).sum()), d[f"{prefix}_tl2"][k] * scale
        if rel:
            assert err <= tol * max(tmax, 1e-6), (prefix, name, err, tmax)
            np.testing.assert_allclose(l2, l2ref, rtol=1e-5, err_msg=f"{prefix} {name}")
        else:
            assert err <= tol, (prefix, name, err)
            assert abs(l2 - l2ref) <= tol * np.sqrt(n), (prefix, name, l2, l2ref)
        off += n
    assert off == got.size


def test_oracle_cnn_update_pinned_at_h512():
    """cnn_update_h512.npz: the reference's whole T/run.py iteration at c3's hidden
    size (CNNBase H = 512; 4 envs x 4 steps, E = 2, M = 2) replayed by the oracle —
    actions bit-exact, returns 1e-5, losses 1e-5 relative, first-minibatch clipped
    gradient (sampled) within 1e-5 of each tensor's max |g|, per-tensor L2 1e-5,
    final parameters within 2e-5."""
    d = golden("cnn_update_h512.npz")
    hidden, N, T, E, Mb = (int(x) for x in d["meta"])
    assert hidden == 512
    shapes = O.cnn_param_shapes(hidden)
    assert [str(n) for n in d["names"]] == [n for n, _ in shapes]
    r = O.run_iteration(d["init_params"], shapes, d["obs_u8"], d["exp_noise"], d["rewards"][..., 0],
                        d["masks"][..., 0], d["perms"], num_mini_batch=Mb, lr=float(d["lr"][0]))
    assert np.array_equal(r["actions"], d["actions"][..., 0])
    np.testing.assert_allclose(r["returns"][:T], d["returns"][:T, :, 0], atol=1e-5)
    np.testing.assert_allclose(r["losses"], d["losses"], rtol=1e-5, atol=1e-7)
    clipf = min(1.0, 0.5 / (float(d["total_norms"][0]) + 1e-6))
    _digest_check(r["first"]["clipped_grad"], d, "mb0_preclip_grad", shapes, 1e-5, scale=clipf)
    _digest_check(r["final_params"], d, "final_params", shapes, 2e-5, rel=False)


def test_oracle_recurrent_update_pinned_at_h256():
    """gru_update_h256.npz: the reference's recurrent PPO.update at c5's hidden size
    (GRU H = 256, V = 14; 8 envs x 16 steps, masks with zeros, E = 2, M = 2) —
    oracle.run_update_recurrent's first-minibatch BPTT gradient (sampled) within
    1e-5 of each tensor's max |g|, per-minibatch losses and total norms 1e-5
    relative, final parameters within 2e-5."""
    d = golden("gru_update_h256.npz")
    hidden, V, N, T, E, Mb = (int(x) for x in d["meta"])
    assert hidden == 256
    clip, vcoef, ecoef = (float(x) for x in d["coefs"])
    shapes = O.cnn_param_shapes(hidden, recurrent=True, vector_obs_len=V)
    assert [str(n) for n in d["names"]] == [n for n, _ in shapes]
    masks = np.concatenate([d["masks0"][None], d["masks"]], 0)[..., 0]
    r = O.run_update_recurrent(d["init_params"], shapes, d["obs_u8"], d["vector_obs"], d["h0"], masks,
                               d["actions"][..., 0], d["action_log_probs"][..., 0], d["value_preds_after"][..., 0],
                               d["returns"][..., 0], d["perms"], num_mini_batch=Mb, clip=clip, value_coef=vcoef,
                               entropy_coef=ecoef, lr=float(d["lr"][0]))
    _digest_check(r["preclip_grads"][0], d, "mb0_preclip_grad", shapes, 1e-5)
    np.testing.assert_allclose(r["mb_losses"], d["mb_losses"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(r["total_norms"], d["total_norms"], rtol=1e-5)
    np.testing.assert_allclose(r["losses"], d["losses"], rtol=1e-5, atol=1e-7)
    _digest_check(r["final_params"], d, "final_params", shapes, 2e-5, rel=False)
