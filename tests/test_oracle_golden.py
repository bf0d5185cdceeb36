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
    d = golden("mlp.npz")
    sh = [("actor.0.weight", (64, 4)), ("actor.0.bias", (64,)), ("actor.2.weight", (64, 64)),
          ("actor.2.bias", (64,)), ("critic.0.weight", (64, 4)), ("critic.0.bias", (64,)),
          ("critic.2.weight", (64, 64)), ("critic.2.bias", (64,)), ("critic_linear.weight", (1, 64)),
          ("critic_linear.bias", (1,))]
    assert [str(n) for n in d["base_names"]] == [n for n, _ in sh]
    p = O.unflatten(d["base_params"], sh)
    x = d["x"].astype(np.float64)

    def mlp(pre):
        h = np.tanh(x @ p[pre + ".0.weight"].T + p[pre + ".0.bias"])
        return np.tanh(h @ p[pre + ".2.weight"].T + p[pre + ".2.bias"])

    value = mlp("critic") @ p["critic_linear.weight"].T + p["critic_linear.bias"]
    feat = mlp("actor")
    np.testing.assert_allclose(value, d["value"], atol=1e-6)
    np.testing.assert_allclose(feat, d["actor_features"], atol=1e-6)
    hp = d["head_params"]
    logits = feat @ hp[:128].reshape(2, 64).T + hp[128:]
    c = O.categorical(logits)
    np.testing.assert_allclose(c["norm_logits"], d["norm_logits"], atol=1e-6)
    np.testing.assert_allclose(c["entropy"], d["entropy"], atol=1e-6)


def test_gru_evaluate_actions():
    d = golden("gru_eval.npz")
    hidden, V, N, T = [int(x) for x in d["meta"]]
    shapes = O.cnn_param_shapes(hidden, recurrent=True, vector_obs_len=V)
    assert [str(n) for n in d["names"]] == [n for n, _ in shapes]
    p = O.unflatten(d["params"], shapes)
    x = O.decode_obs(d["obs_u8"].reshape(T * N, 4, 84, 84))
    feat, _ = O.cnn_trunk(p, x)
    xin = np.concatenate([feat, d["vector_obs"].reshape(T * N, V)], 1)
    out, hT = O.gru_sequence(p, xin, d["h0"], d["masks"])
    value = out @ p["base.critic_linear.weight"].T + p["base.critic_linear.bias"]
    c = O.categorical(out @ p["dist.linear.weight"].T + p["dist.linear.bias"])
    logp = np.take_along_axis(c["norm_logits"], d["actions"], -1)
    np.testing.assert_allclose(value, d["values"], atol=2e-6)
    np.testing.assert_allclose(logp, d["log_probs"], atol=2e-6)
    np.testing.assert_allclose(c["entropy"].mean(), d["entropy"][0], atol=2e-6)
    np.testing.assert_allclose(hT, d["hT"], atol=2e-6)


def test_full_iteration_replay():
    """One T/run.py iteration replayed through the oracle matches the reference."""
    d = golden("cnn_update.npz")
    hidden, N, T, E, Mb = [int(x) for x in d["meta"]]
    shapes = O.cnn_param_shapes(hidden)
    assert [str(n) for n in d["names"]] == [n for n, _ in shapes]
    r = O.run_iteration(d["init_params"], shapes, d["obs_u8"], d["exp_noise"], d["rewards"][..., 0],
                        d["masks"][..., 0], d["perms"], num_mini_batch=Mb, lr=float(d["lr"][0]))
    assert np.array_equal(r["actions"], d["actions"][..., 0])
    np.testing.assert_allclose(r["values"], d["values"][..., 0], atol=1e-6)
    np.testing.assert_allclose(r["log_probs"], d["action_log_probs"][..., 0], atol=1e-6)
    np.testing.assert_allclose(r["returns"], d["returns"][..., 0], atol=1e-6)
    np.testing.assert_allclose(r["first"]["clipped_grad"], d["mb0_clipped_grad"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(r["losses"], d["losses"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r["final_params"], d["final_params"], rtol=0, atol=1e-6)


def test_gru_backward_finite_difference():
    """The oracle's hand-written BPTT (used to check the HIP GRU backward) against
    central finite differences of its own forward (float64)."""
    rng = np.random.default_rng(0)
    H, I, T, n = 4, 3, 5, 2
    p = {"base.gru.weight_ih_l0": rng.standard_normal((3 * H, I)) * 0.5,
         "base.gru.weight_hh_l0": rng.standard_normal((3 * H, H)) * 0.5,
         "base.gru.bias_ih_l0": rng.standard_normal(3 * H) * 0.1,
         "base.gru.bias_hh_l0": rng.standard_normal(3 * H) * 0.1}
    x = rng.standard_normal((T * n, I))
    h0 = rng.standard_normal((n, H))
    masks = (rng.random((T, n)) > 0.3).astype(np.float64)
    wout = rng.standard_normal((T * n, H))

    def loss(pp, xx):
        out, _ = O.gru_sequence_cache(pp, xx, h0, masks)
        return (out * wout).sum()

    out, cache = O.gru_sequence_cache(p, x, h0, masks)
    g, dx = O.gru_backward(p, x, masks, cache, wout)
    eps = 1e-6
    for k in p:
        num = np.zeros_like(p[k])
        for i in np.ndindex(p[k].shape):
            pp = {kk: v.copy() for kk, v in p.items()}
            pp[k][i] += eps
            lp = loss(pp, x)
            pp[k][i] -= 2 * eps
            num[i] = (lp - loss(pp, x)) / (2 * eps)
        np.testing.assert_allclose(g[k], num, rtol=1e-5, atol=1e-7)
    num = np.zeros_like(x)
    for i in np.ndindex(x.shape):
        xx = x.copy()
        xx[i] += eps
        lp = loss(p, xx)
        xx[i] -= 2 * eps
        num[i] = (lp - loss(p, xx)) / (2 * eps)
    np.testing.assert_allclose(dx, num, rtol=1e-5, atol=1e-7)
