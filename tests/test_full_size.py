"""Full-size parity (BASELINE.json configs c2, c3, c5 at their own shapes): one
whole rollout of the drop-in API on the synthetic env, then

  * returns bit-exact vs the C oracle of compute_returns (storage.py:82-121) on
    the storage that rollout produced, advantage statistics vs the oracle;
  * stored values / log-probs on a strided subset vs the float64 forward;
  * one full minibatch gradient (c3: 65,536 rows, c2: 16,384 rows) vs float64
    autograd of the reference's loss (oracle/torch_ref.py: algo/ppo.py:57-81 with
    torch.distributions.Categorical, convolutions as explicit im2col GEMMs in
    float64 on the GPU), 1e-5 of each tensor's max |g|, losses 2e-5 relative;
  * c5: one 512-env x 256-step recurrent minibatch (H=256, V=14): the GRU, head
    and trunk gradients vs float64 — the oracle's BPTT (oracle.gru_backward) on the
    engine's own GRU inputs, and float64 autograd of the trunk driven by the
    oracle's dL/dx — 1e-5 of each tensor's max |g|.

These take seconds to minutes on the MI355X; the float64 references run on the
GPU (torch) and on the host (numpy, GRU only)."""
import numpy as np
import pytest
import torch

from oracle import ppo_oracle as O
from oracle import torch_ref as TR
from helpers.gradcheck import check_grads as _check_grads

pytestmark = pytest.mark.gpu

HP = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.001, "use_clipped_value_loss": True}


class _GradCapture(object):
    """FlatAdam stand-in: keeps the minibatch's flat gradient (no parameter step)."""

    def _step_flat(self, eng):
        self.grad = eng.grad.clone()


def _rollout(pol, st, env, T, vec=None):
    for step in range(T):
        with torch.no_grad():
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step], st.masks[step])
        r, m, bm = env.step_into(st.obs[step + 1], a)
        st.insert(st.obs[step + 1], vec if vec is not None else st.vector_obs[step + 1], h, a, lp, v, r, m, bm)
    with torch.no_grad():
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
    return nv


def _check_returns(st, nv):
    """compute_returns bit-exact vs the C oracle on this storage; advantage
    statistics vs the oracle's (ppo.py:35-37)."""
    r = st.rewards[..., 0].cpu().numpy()
    v = st.value_preds[..., 0].cpu().numpy().copy()
    m = st.masks[..., 0].cpu().numpy()
    bm = st.bad_masks[..., 0].cpu().numpy()
    st.compute_returns(nv, True, 0.99, 0.95, False)
    eret, ev = O.compute_returns(r, v, m, bm, nv.reshape(-1).cpu().numpy(), True, 0.99, 0.95, False)
    T = r.shape[0]
    assert np.array_equal(st.returns[:T, :, 0].cpu().numpy(), eret[:T])
    assert np.array_equal(st.value_preds[..., 0].cpu().numpy(), ev)
    adv = st.normalized_advantages()
    ref = O.normalize_advantages(eret, ev)
    np.testing.assert_allclose(adv.cpu().numpy(), ref, rtol=1e-6, atol=1e-6)
    mean, std = O.adv_stats(eret, ev)
    stats = st._adv_stats.cpu().numpy()
    assert stats[0] == st.rewards.numel()   # {count, mean, M2} (Welford / Chan)
    np.testing.assert_allclose(stats[1], mean, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(np.sqrt(stats[2] / (stats[0] - 1)), std, rtol=1e-5)
    return adv


def _engine_relu_masks(eng, B, H):
    """the ReLU decisions of the engine's training forward of the minibatch just run
    (its workspace activations a1..a3 and fc output h, NHWC -> the reference's NCHW)"""
    bufs = eng.ws["train"].bufs
    a1 = bufs["a1"][:B * 12800].view(B, 20, 20, 32).permute(0, 3, 1, 2)
    a2 = bufs["a2"][:B * 5184].view(B, 9, 9, 64).permute(0, 3, 1, 2)
    a3 = bufs["a3"][:B * 1568].view(B, 7, 7, 32).permute(0, 3, 1, 2)
    h = bufs["h"][:B * H].view(B, H)
    return [t > 0 for t in (a1, a2, a3, h)]


def _check_relu_decisions(p, obs_in, ridx, masks, chunk=4096, rel=1e-5):
    """every ReLU decision of the engine agrees with float64's, except where the
    float64 pre-activation is within rel x that layer's max |pre-activation| of 0;
    returns the number of such flips per layer"""
    w1, b1, w2, b2, w3, b3, w4, b4 = [t.detach() for t in p[:8]]
    B = masks[0].shape[0]
    flips, worst, zmax = [0] * 4, [0.0] * 4, [0.0] * 4
    with torch.no_grad():
        for s in range(0, B, chunk):
            e = min(B, s + chunk)
            rows = slice(s, e) if ridx is None else ridx[s:e].to(obs_in.device)
            x = TR._decode(obs_in[rows], w1.device, torch.float64)
            z1 = TR.conv_unfold(x, w1, b1, 4)
            z2 = TR.conv_unfold(torch.relu(z1), w2, b2, 2)
            z3 = TR.conv_unfold(torch.relu(z2), w3, b3, 1)
            z4 = torch.nn.functional.linear(torch.relu(z3).reshape(e - s, -1), w4, b4)
            for k, z in enumerate((z1, z2, z3, z4)):
                d = (z > 0) != masks[k][s:e]
                zmax[k] = max(zmax[k], z.abs().max().item())
                if d.any():
                    flips[k] += int(d.sum())
                    worst[k] = max(worst[k], z[d].abs().max().item())
    for k in range(4):
        assert worst[k] <= rel * zmax[k], (k, flips, worst, zmax)
    return flips


def _obs_setup(kind, N, T, gpu, pol, env):
    """storage + env-step writer for an observation form (bench.py --obs):
    u8 — synthetic u8 4x84x84 frames (the headline); f32 — the reference's fp32
    storage plane, filled by the f2 chain from raw RGB frames (ppo_obs_preprocess);
    rgb — the raw RGB frames stored, the same decode fused into conv1.  Returns
    (storage, write(slot, action|None), decode(rows of the obs plane) -> fp32 x)."""
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.vec_env import ObsPreprocess
    if kind == "u8":
        st = RolloutStorage(T, N, (4, 84, 84), [0], env.action_space, 1, obs_dtype=torch.uint8, device=gpu)
        write = lambda slot, a=None: env.step_into(slot, a) if a is not None else env.reset_into(slot)  # noqa: E731
        return st, write, lambda rows: rows.double() / 255.0
    mean = np.random.default_rng(0).uniform(20, 80, (84, 84, 3)).astype(np.float32).astype(np.float64)
    pre = ObsPreprocess(84, "norm", mean, 36.31282043457031, device=gpu)
    if kind == "rgb":
        pol.set_obs_decode(pre)
        st = RolloutStorage(T, N, (84, 84, 3), [0], env.action_space, 1, obs_dtype=torch.uint8, device=gpu)
        write = lambda slot, a=None: env.step_into(slot, a) if a is not None else env.reset_into(slot)  # noqa: E731
        return st, write, lambda rows: pre(rows.contiguous())
    st = RolloutStorage(T, N, (4, 84, 84), [0], env.action_space, 1, obs_dtype=torch.float32, device=gpu)
    raw = torch.empty(N, 84, 84, 3, dtype=torch.uint8, device=gpu)

    def write(slot, a=None):
        out = env.step_into(raw, a) if a is not None else env.reset_into(raw)
        pre(raw, out=slot)
        return out
    return st, write, lambda rows: rows


@pytest.mark.parametrize("N,kind", [(4096, "u8"), (1024, "u8"), (4096, "f32"), (4096, "rgb")])   # c3, c2 (T=128, 8 minibatches)
def test_cnn_iteration_full_size(gpu, N, kind):
    """kind f32 / rgb: the observation forms the reference's own env chain hands
    over (fp32 storage plane; raw RGB frames with the decode fused into conv1),
    held to the same bar as the u8 headline path."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    T, H, Mb = 128, 512, 8
    torch.manual_seed(1)
    env = SyntheticVecEnv(N, obs_shape=(4, 84, 84) if kind == "u8" else (84, 84, 3), seed=123, p_done=0.01,
                          device=gpu)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    flat0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    pol.to(gpu)
    st, write, decode = _obs_setup(kind, N, T, gpu, pol, env)
    write(st.obs[0])
    for step in range(T):
        with torch.no_grad():
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step], st.masks[step])
        r, m, bm = write(st.obs[step + 1], a)
        st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, r, m, bm)
    with torch.no_grad():
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
    torch.cuda.synchronize()

    # stored values / log-probs of the rollout vs the float64 forward (strided subset)
    shapes = O.cnn_param_shapes(H)
    p64 = O.unflatten(flat0.numpy(), shapes)
    ts, ns = np.array([0, T // 2, T - 1]), np.arange(0, N, 64)
    rows = st.obs[ts][:, ns].reshape(len(ts) * len(ns), *st.obs.shape[2:])
    value, logits, _ = O.cnn_forward(p64, decode(rows).double().cpu().numpy())
    c = O.categorical(logits)
    acts = st.actions[ts][:, ns].cpu().numpy().reshape(-1)
    lp_ref = np.take_along_axis(c["norm_logits"], acts[:, None], 1)[:, 0]
    np.testing.assert_allclose(st.value_preds[ts][:, ns].cpu().numpy().reshape(-1), value, atol=1e-4)
    np.testing.assert_allclose(st.action_log_probs[ts][:, ns].cpu().numpy().reshape(-1), lp_ref, atol=1e-4)

    adv = _check_returns(st, nv)

    # the first minibatch of the update: its gradient vs float64 autograd
    eng = pol.hip_engine()
    B = N * T // Mb
    idx = torch.randperm(N * T)[:B].to(gpu)
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)
    cap = _GradCapture()
    eng.train_minibatch(st, adv, idx, HP, loss, cap)
    torch.cuda.synchronize()
    flat = lambda t: t[:T].reshape(T * N, *t.shape[2:])  # noqa: E731
    if kind == "u8":
        obs_in, planes, ridx = flat(st.obs), [flat(st.actions), flat(st.action_log_probs), adv.reshape(-1),
                                              flat(st.value_preds), flat(st.returns)], idx
    else:   # the minibatch's fp32 policy input (the reference chain's values), rows in minibatch order
        obs_in = decode(flat(st.obs)[idx])
        planes = [flat(st.actions)[idx], flat(st.action_log_probs)[idx], adv.reshape(-1)[idx],
                  flat(st.value_preds)[idx], flat(st.returns)[idx]]
        ridx = None
    p = TR.unflatten(flat0, H, dtype=torch.float64, device=gpu, requires_grad=True)
    # both references take the engine's ReLU decisions, each checked first against
    # float64's own: they may differ only where float64's pre-activation is within
    # rounding of 0 (a flip there moves a gradient by a whole row's term — at c2's
    # 16,384 rows one fc flip is ~3e-6 of the fc bias gradient, which made the
    # comparison a coin toss on summation order); the gradients then measure arithmetic
    masks = _engine_relu_masks(eng, B, H)
    print("ReLU decisions differing from float64's:", _check_relu_decisions(p, obs_in, ridx, masks), flush=True)
    grads, losses = TR.minibatch_grads(p, obs_in, *planes, idx=ridx, clip=HP["clip"], value_coef=HP["value_coef"],
                                       entropy_coef=HP["entropy_coef"], masks=masks)
    print("float64 reference done", flush=True)
    # the same gradient at the reference's precision: torch fp32 autograd on the
    # device (im2col GEMMs on the vendor BLAS, chunk gradients summed in fp32)
    p32 = TR.unflatten(flat0, H, dtype=torch.float32, device=gpu, requires_grad=True)
    g32, _ = TR.minibatch_grads(p32, obs_in, *planes, idx=ridx, chunk=8192, clip=HP["clip"],
                                value_coef=HP["value_coef"], entropy_coef=HP["entropy_coef"], masks=masks)
    print("fp32 comparator done", flush=True)
    g32 = torch.cat([t.reshape(-1) for t in g32]).cpu().numpy()
    _check_grads(cap.grad.cpu().numpy(), grads, shapes, fp32_flat=g32)
    np.testing.assert_allclose(loss[:3].cpu().numpy(), losses, rtol=2e-5, atol=1e-7)
    assert loss[3].item() == 0


def test_recurrent_minibatch_full_size(gpu):
    """c5: GRU H=256 + 14 vector obs; one recurrent_generator minibatch of 512
    envs x 256 steps (131,072 rows) from a 1024-lane rollout."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    N, T, H, V, n = 1024, 256, 256, 14, 512
    torch.manual_seed(2)
    env = SyntheticVecEnv(N, seed=321, p_done=0.01, device=gpu)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
                   vector_obs_len=V)
    flat0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    pol.to(gpu)
    st = RolloutStorage(T, N, (4, 84, 84), [V], env.action_space, H, obs_dtype=torch.uint8, device=gpu)
    env.reset_into(st.obs[0])
    vec = torch.rand(N, V, generator=torch.Generator().manual_seed(3)).to(gpu)
    st.vector_obs[0].copy_(vec)
    nv = _rollout(pol, st, env, T, vec=vec)
    torch.cuda.synchronize()
    adv = _check_returns(st, nv)

    eng = pol.hip_engine()
    envs = torch.randperm(N)[:n].to(gpu)
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)
    cap = _GradCapture()
    eng.train_minibatch_rec(st, adv, envs, HP, loss, cap)
    torch.cuda.synchronize()
    R = T * n
    I, Ip = H + V, eng.Ip
    x = eng.ws["train"].bufs["xpad"][:R * Ip].reshape(R, Ip)[:, :I].double().cpu().numpy()   # the GRU inputs used
    ev = envs.cpu().numpy()
    rows = (np.arange(T)[:, None] * N + ev[None, :]).reshape(-1)                             # row t*n + j
    # the engine's GRU inputs are fc(obs) | vector obs: check them against float64 first
    shapes = O.cnn_param_shapes(H, recurrent=True, vector_obs_len=V)
    names = [nm for nm, _ in shapes]
    p64 = O.unflatten(flat0.numpy(), shapes)
    trunk_p = [torch.tensor(p64[nm], device=gpu, requires_grad=True) for nm in names[4:12]]
    obs_flat = st.obs[:T].reshape(T * N, 4, 84, 84)
    ridx = torch.from_numpy(rows).to(gpu)
    sub = np.arange(0, R, 97)
    with torch.no_grad():
        feat = TR.trunk(trunk_p, obs_flat[ridx[sub]].double() / 255.0, TR.conv_unfold).cpu().numpy()
    np.testing.assert_allclose(x[sub, :H], feat, rtol=0, atol=2e-5 * max(1.0, np.abs(feat).max()))
    np.testing.assert_array_equal(x[:, H:], st.vector_obs[:T].reshape(T * N, V).cpu().numpy()[rows].astype(np.float64))
    # float64 GRU + heads + loss (oracle), BPTT to dL/dx
    h0 = st.recurrent_hidden_states[0].cpu().numpy()[ev].astype(np.float64)
    masks = st.masks[:T, :, 0].cpu().numpy()[:, ev].astype(np.float64)
    out, gcache = O.gru_sequence_cache(p64, x, h0, masks)
    value, logits = O.heads(p64, out)
    f = lambda t: t[:T].reshape(-1).cpu().numpy()[rows]  # noqa: E731
    lg = O.loss_head_grads(value, logits, f(st.actions), f(st.action_log_probs), adv.reshape(-1).cpu().numpy()[rows],
                           f(st.value_preds), f(st.returns), HP["clip"], HP["value_coef"], HP["entropy_coef"])
    g = {"base.critic_linear.weight": lg["g_value"][None, :] @ out,
         "base.critic_linear.bias": np.array([lg["g_value"].sum()]),
         "dist.linear.weight": lg["g_logits"].T @ out, "dist.linear.bias": lg["g_logits"].sum(0)}
    dout = lg["g_value"][:, None] * p64["base.critic_linear.weight"] + lg["g_logits"] @ p64["dist.linear.weight"]
    gg, dx = O.gru_backward(p64, x, masks, gcache, dout)
    g.update(gg)
    tg = TR.trunk_grads(trunk_p, obs_flat, torch.from_numpy(dx[:, :H]).to(gpu), idx=ridx)
    for nm, t in zip(names[4:12], tg):
        g[nm] = t.cpu().numpy()
    _check_grads(cap.grad.cpu().numpy(), [g[nm] for nm in names], shapes)
    np.testing.assert_allclose(loss[:3].cpu().numpy(), [lg["value_loss"], lg["action_loss"], lg["entropy"]],
                               rtol=2e-5, atol=1e-7)


def test_recurrent_rollout_4096_lanes(gpu):
    """c5's rollout width: 4096 lanes of GRU acting (H=256, V=14, episode ends
    resetting the hidden state through masks) for 24 steps.  On a strided subset
    of lanes the stored values, log-probs of the sampled actions and hidden states
    vs the float64 forward (trunk -> GRU sequence with the stored masks ->
    heads: model.py:116-165, 185-188; oracle.gru_sequence)."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    N, T, H, V = 4096, 24, 256, 14
    torch.manual_seed(5)
    env = SyntheticVecEnv(N, seed=77, p_done=0.05, device=gpu)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
                   vector_obs_len=V)
    flat0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    pol.to(gpu)
    st = RolloutStorage(T, N, (4, 84, 84), [V], env.action_space, H, obs_dtype=torch.uint8, device=gpu)
    env.reset_into(st.obs[0])
    vec = torch.rand(N, V, generator=torch.Generator().manual_seed(8)).to(gpu)
    st.vector_obs[0].copy_(vec)
    _rollout(pol, st, env, T, vec=vec)
    torch.cuda.synchronize()
    masks = st.masks[:T, :, 0].cpu().numpy()
    assert (masks == 0).sum() > 0                   # some lanes reset their hidden state
    shapes = O.cnn_param_shapes(H, recurrent=True, vector_obs_len=V)
    names = [nm for nm, _ in shapes]
    p64 = O.unflatten(flat0.numpy(), shapes)
    trunk_p = [torch.tensor(p64[nm], device=gpu) for nm in names[4:12]]
    ns = np.arange(3, N, 61)
    nsg = torch.from_numpy(ns).to(gpu)
    with torch.no_grad():
        obs = st.obs[:T][:, nsg].reshape(T * len(ns), 4, 84, 84)
        feat = TR.trunk(trunk_p, obs.double() / 255.0, TR.conv_unfold).cpu().numpy()
    x = np.concatenate([feat, np.broadcast_to(vec.cpu().numpy()[ns].astype(np.float64), (T, len(ns), V))
                        .reshape(T * len(ns), V)], 1)
    h0 = st.recurrent_hidden_states[0].cpu().numpy()[ns].astype(np.float64)
    out, _ = O.gru_sequence(p64, x, h0, masks[:, ns].astype(np.float64))
    value, logits = O.heads(p64, out)
    acts = st.actions[:T][:, nsg].cpu().numpy().reshape(-1)
    lp_ref = np.take_along_axis(O.categorical(logits)["norm_logits"], acts[:, None], 1)[:, 0]
    np.testing.assert_allclose(st.recurrent_hidden_states[1:T + 1][:, nsg].cpu().numpy().reshape(-1, H),
                               out, atol=1e-4)
    np.testing.assert_allclose(st.value_preds[:T][:, nsg].cpu().numpy().reshape(-1), value, atol=1e-4)
    np.testing.assert_allclose(st.action_log_probs[:T][:, nsg].cpu().numpy().reshape(-1), lp_ref, atol=1e-4)
