#!/usr/bin/env python3
"""Golden-vector generator — CONTAINER ONLY, never shipped to the GPU box.

Imports the reference's own hot-path modules from /root/reference (read-only)
and records their outputs on seeded inputs into tests/golden/*.npz.  The
fixtures are data (inputs + expected outputs); no reference source is copied.

Reference modules used (SURVEY.md §8c "How to import"):
  * B/ = ppo-dash-study/001_baseline/ppo/{storage,model,distributions}.py and
    ppo/algo/ppo.py — the vector-less CNN variant (T/ crashes when V=0,
    T/a2c_ppo_acktr/storage.py:144).
  * T/ = ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/... — the
    recurrent (GRU) + vector-obs variant.
A stub `<pkg>.envs` module stands in for the gym/baselines-backed envs.py,
which only provides the VecNormalize type to utils.py.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [name ...]
      (names: gae advnorm sampler categorical cnn_update cnn_update_h512
       cnn_update_wide adam mlp gru gru_update gru_update_h256; none = all)
"""
import importlib
import importlib.util
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import torch  # noqa: E402

# distributions.py patches torch.distributions.Categorical.sample in place
# (sample = old_sample(self).unsqueeze(-1)); importing a second reference tree
# would wrap the wrapper, so each load starts from torch's own method
_TORCH_CAT_SAMPLE = torch.distributions.Categorical.sample

REF_ROOT = "/root/reference"
B_DIR = f"{REF_ROOT}/ppo-dash-study/001_baseline"
T_DIR = f"{REF_ROOT}/ppo-dash-training/pytorch-a2c-ppo-acktr-gail"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


class Discrete:  # duck-typed gym.spaces.Discrete (storage.py:20, model.py:30)
    def __init__(self, n):
        self.n = n


def load_ref(variant):
    """Import (storage, model, distributions, ppo) of one reference tree."""
    ref, pkg = (B_DIR, "ppo") if variant == "B" else (T_DIR, "a2c_ppo_acktr")
    for k in list(sys.modules):
        if k == pkg or k.startswith(pkg + "."):
            del sys.modules[k]
    while ref in sys.path:
        sys.path.remove(ref)
    for other in (B_DIR, T_DIR):
        while other in sys.path:
            sys.path.remove(other)
    sys.path.insert(0, ref)
    torch.distributions.Categorical.sample = _TORCH_CAT_SAMPLE
    stub = types.ModuleType(pkg + ".envs")
    stub.VecNormalize = type("VecNormalize", (), {})
    sys.modules[pkg + ".envs"] = stub
    S = importlib.import_module(pkg + ".storage")
    M = importlib.import_module(pkg + ".model")
    D = importlib.import_module(pkg + ".distributions")
    spec = importlib.util.spec_from_file_location(f"refppo_{variant}", f"{ref}/{pkg}/algo/ppo.py")
    P = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(P)
    return S, M, D, P


def flat_params(module):
    return np.concatenate([p.detach().reshape(-1).numpy().astype(np.float32)
                           for p in module.parameters()])


def param_names(module):
    return np.array([n for n, _ in module.named_parameters()])


def digest(prefix, flat, module, stride):
    """A production-size tensor in a small fixture: every stride-th element (global
    index), and per parameter tensor its max |x| and L2 norm (float64)."""
    idx = np.arange(0, flat.size, stride, dtype=np.int64)
    tmax, tl2, off = [], [], 0
    for p in module.parameters():
        seg = flat[off:off + p.numel()].astype(np.float64)
        tmax.append(np.abs(seg).max())
        tl2.append(np.sqrt((seg * seg).sum()))
        off += p.numel()
    return {f"{prefix}_idx": idx, f"{prefix}_sampled": flat[idx], f"{prefix}_tmax": np.array(tmax),
            f"{prefix}_tl2": np.array(tl2)}


def sample_margin(pol, obs, vec, hxs, masks, En):
    """min over rows of the relative gap between the two largest probs / E (the
    multinomial draw's argmax): a replay whose probabilities differ by
    fp32 rounding picks the same actions when this is well above 1e-6"""
    with torch.no_grad():
        _, feats, _ = pol.base(obs, vec, hxs, masks)
        q = (pol.dist(feats).probs / En).double()
    top = torch.topk(q, 2, dim=1).values
    return float(((top[:, 0] - top[:, 1]) / top[:, 0]).min())


def save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path}  ({os.path.getsize(path) / 1024:.1f} KiB)")


# ---------------------------------------------------------------------------
# (1) GAE / returns, all four compute_returns branches (storage.py:82-121)
# ---------------------------------------------------------------------------
def gen_gae(S):
    out = {}
    rng = np.random.default_rng(7)
    T, N = 32, 64
    r = rng.standard_normal((T, N, 1)).astype(np.float32)
    v = (3.0 * rng.standard_normal((T + 1, N, 1))).astype(np.float32)
    m = (rng.random((T + 1, N, 1)) < 0.95).astype(np.float32)
    bm = (rng.random((T + 1, N, 1)) < 0.95).astype(np.float32)
    nv = (3.0 * rng.standard_normal((N, 1))).astype(np.float32)
    out.update(rewards=r, value_preds=v, masks=m, bad_masks=bm, next_value=nv)
    for gi, (gamma, lam) in enumerate([(0.99, 0.95), (0.997, 0.9)]):
        for use_gae in (True, False):
            for ptl in (True, False):
                st = S.RolloutStorage(T, N, (1,), [0], Discrete(2), 1)
                st.rewards.copy_(torch.from_numpy(r))
                st.value_preds.copy_(torch.from_numpy(v))
                st.masks.copy_(torch.from_numpy(m))
                st.bad_masks.copy_(torch.from_numpy(bm))
                st.returns.fill_(-7.0)  # sentinel: GAE branches leave returns[T] untouched
                st.compute_returns(torch.from_numpy(nv), use_gae, gamma, lam, ptl)
                key = f"g{gi}_gae{int(use_gae)}_ptl{int(ptl)}"
                out[key + "_returns"] = st.returns.numpy().copy()
                out[key + "_value_preds"] = st.value_preds.numpy().copy()
    out["gammas"] = np.array([0.99, 0.997])
    out["lambdas"] = np.array([0.95, 0.9])
    save("gae.npz", **out)


# ---------------------------------------------------------------------------
# (2) advantage normalisation as PPO.update computes it (ppo.py:35-37)
#     captured by intercepting the `advantages` handed to the generator
# ---------------------------------------------------------------------------
def gen_advnorm(S, P):
    out = {}
    for ci, (T, N, scale) in enumerate([(32, 64, 3.0), (128, 256, 10.0), (7, 5, 1.0)]):
        rng = np.random.default_rng(100 + ci)
        st = S.RolloutStorage(T, N, (1,), [0], Discrete(2), 1)
        ret = (scale * rng.standard_normal((T + 1, N, 1)) + 1.5).astype(np.float32)
        val = (scale * rng.standard_normal((T + 1, N, 1))).astype(np.float32)
        st.returns.copy_(torch.from_numpy(ret))
        st.value_preds.copy_(torch.from_numpy(val))
        captured = []

        def fake_gen(advantages, num_mini_batch, _c=captured):
            _c.append(advantages.clone())
            return iter(())

        st.feed_forward_generator = fake_gen

        class _AC:
            is_recurrent = False

            def parameters(self):
                return [torch.nn.Parameter(torch.zeros(1))]

        agent = P.PPO(_AC(), 0.1, 1, 1, 0.5, 0.001, lr=1e-4, eps=1e-5, max_grad_norm=0.5)
        agent.update(st)
        out[f"c{ci}_returns"] = ret
        out[f"c{ci}_value_preds"] = val
        out[f"c{ci}_advantages"] = captured[0].numpy()
    save("advnorm.npz", **out)


# ---------------------------------------------------------------------------
# (3) minibatch samplers (storage.py:123-223): indices recovered from a
#     storage whose value_preds hold their own flat row index t*N+n
# ---------------------------------------------------------------------------
def gen_sampler(S):
    out = {}
    cases = [(0, 16, 8, 4), (1, 128, 32, 8), (1234, 64, 7, 3), (5, 128, 1024 // 128 * 4, 8)]
    for ci, (seed, T, N, M) in enumerate(cases):
        st = S.RolloutStorage(T, N, (1,), [0], Discrete(2), 1)
        st.value_preds[:-1].copy_(torch.arange(T * N, dtype=torch.float32).view(T, N, 1))
        adv = torch.zeros(T, N, 1)
        torch.manual_seed(seed)
        ff = [b[4].view(-1).long().numpy().copy() for b in st.feed_forward_generator(adv, M)]
        out[f"c{ci}_meta"] = np.array([seed, T, N, M])
        out[f"c{ci}_ff"] = np.stack(ff).astype(np.int64)
        if N % M == 0:  # recurrent_generator indexes past perm otherwise (storage.py:181-182)
            torch.manual_seed(seed)
            rec = [b[4].view(-1).long().numpy().copy() for b in st.recurrent_generator(adv, M)]
            out[f"c{ci}_rec"] = np.stack(rec).astype(np.int64)
    save("sampler.npz", **out)


# ---------------------------------------------------------------------------
# (4) Categorical head: linear → FixedCategorical → sample/mode/log_probs/
#     entropy (distributions.py:17-27,54-68); Exp(1) noise replayed from the
#     generator state so argmax(probs/E) can be checked bit-exactly
# ---------------------------------------------------------------------------
def gen_categorical(D):
    out = {}
    torch.manual_seed(3)
    Nrow, Hd, A = 4096, 16, 8
    head = D.Categorical(Hd, A)
    # gain-0.01 init makes near-uniform probs; widen the spread so that
    # sampling is non-trivial, still through the module's own forward
    with torch.no_grad():
        head.linear.weight.mul_(150.0)
        head.linear.bias.uniform_(-0.5, 0.5)
    feats = torch.randn(Nrow, Hd)
    with torch.no_grad():
        dist = head(feats)
        st = torch.get_rng_state()
        action = dist.sample()
        st_after = torch.get_rng_state()
        torch.set_rng_state(st)
        E = torch.empty(Nrow, A).exponential_(1)
        assert torch.equal(torch.get_rng_state(), st_after), "sample consumed more than one exponential_ draw"
        logp = dist.log_probs(action)
        ent = dist.entropy()
        mode = dist.mode()
    out.update(features=feats.numpy(), weight=head.linear.weight.detach().numpy(),
               bias=head.linear.bias.detach().numpy(), logits_raw=(feats @ head.linear.weight.t() + head.linear.bias).detach().numpy(),
               norm_logits=dist.logits.numpy(), probs=dist.probs.numpy(), exp_noise=E.numpy(),
               action=action.numpy().astype(np.int64), log_probs=logp.numpy(),
               entropy=ent.numpy(), mode=mode.numpy().astype(np.int64))
    save("categorical.npz", **out)


# ---------------------------------------------------------------------------
# (5) one full CNN iteration, run.py:134-248 ordering:
#     act → env → insert ×T, get_value, compute_returns, update, after_update
# ---------------------------------------------------------------------------
def gen_cnn_update(S, M, P, *, hidden, N, T, E, Mb, lr, fname, lowres=False, stride=0, obs_seed=None):
    """lowres: 21x21 random bytes upsampled x4 (a compressible fixture); stride > 0:
    final parameters and gradients as digests (every stride-th element + per-tensor
    max |x| and L2, `digest`); obs_seed: observations not stored but drawn up front as
    torch.randint(0, 256, (T+1, N, 4, 84, 84), generator=Generator().manual_seed(obs_seed))
    — the CPU generator is deterministic, so the replay regenerates them (checked by
    the stored byte sum and CRC-32)"""
    torch.manual_seed(1)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase,
                   base_kwargs={"recurrent": False, "hidden_size": hidden}, vector_obs_len=0)
    agent = P.PPO(pol, 0.1, E, Mb, 0.5, 0.001, lr=lr, eps=1e-5, max_grad_norm=0.5)
    st = S.RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), pol.recurrent_hidden_state_size)
    init = flat_params(pol)
    rng_init = torch.get_rng_state().numpy().copy()
    genv = torch.Generator().manual_seed(123)
    all_obs = None
    if obs_seed is not None:
        all_obs = torch.randint(0, 256, (T + 1, N, 4, 84, 84), dtype=torch.uint8,
                                generator=torch.Generator().manual_seed(obs_seed))

    def frame(k):
        if all_obs is not None:
            return all_obs[k]
        if lowres:
            lo = torch.randint(0, 256, (N, 4, 21, 21), dtype=torch.uint8, generator=genv)
            return lo.repeat_interleave(4, 2).repeat_interleave(4, 3).contiguous()
        return torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, generator=genv)

    obs_u8 = np.zeros((T + 1, N, 4, 84, 84), np.uint8)
    o0 = frame(0)
    obs_u8[0] = o0.numpy()
    st.obs[0].copy_(o0.float() / 255.0)
    noise, values, actions, logps, rewards, masks = [], [], [], [], [], []
    margin = 1.0
    for step in range(T):
        with torch.no_grad():
            rs = torch.get_rng_state()
            value, action, logp, hxs = pol.act(st.obs[step], st.vector_obs[step],
                                               st.recurrent_hidden_states[step], st.masks[step])
            after = torch.get_rng_state()
            torch.set_rng_state(rs)
            En = torch.empty(N, 8).exponential_(1)
            assert torch.equal(torch.get_rng_state(), after)
            torch.set_rng_state(after)
        margin = min(margin, sample_margin(pol, st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                           st.masks[step], En))
        o = frame(step + 1)
        rew = torch.rand(N, 1, generator=genv)
        done = torch.rand(N, generator=genv) < 0.3
        mk = torch.FloatTensor([[0.0] if d else [1.0] for d in done])
        bmk = torch.ones(N, 1)
        obs_u8[step + 1] = o.numpy()
        st.insert(o.float() / 255.0, torch.zeros(N, 0), hxs, action, logp, value, rew, mk, bmk)
        noise.append(En.numpy()); values.append(value.numpy()); actions.append(action.numpy())
        logps.append(logp.numpy()); rewards.append(rew.numpy()); masks.append(mk.numpy())
    print(f"{fname}: min relative sampling margin {margin:.3e}")
    with torch.no_grad():
        next_value = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1],
                                   st.masks[-1]).detach()
    st.compute_returns(next_value, True, 0.99, 0.95, False)
    returns = st.returns.numpy().copy()
    vpreds = st.value_preds.numpy().copy()

    # capture: minibatch permutations (replayed from the generator state),
    # the first minibatch's outputs and clipped grads, the loss triple
    rng_before_update = torch.get_rng_state()
    mb_records = []
    orig_eval = pol.evaluate_actions

    def eval_wrap(*a, **k):
        res = orig_eval(*a, **k)
        mb_records.append({"values": res[0].detach().numpy().copy(),
                           "logp": res[1].detach().numpy().copy(),
                           "entropy": float(res[2].detach())})
        return res

    pol.evaluate_actions = eval_wrap
    grads = []
    orig_step = agent.optimizer.step

    def step_wrap(*a, **k):
        grads.append(np.concatenate([p.grad.reshape(-1).numpy().copy() for p in pol.parameters()]))
        return orig_step(*a, **k)

    agent.optimizer.step = step_wrap
    preclip, norms = [], []
    orig_clip = torch.nn.utils.clip_grad_norm_

    def clip_wrap(params, max_norm, *a, **k):   # clip_grad_norm_'s input and total norm
        params = list(params)
        preclip.append(np.concatenate([q.grad.reshape(-1).numpy().copy() for q in params]))
        tn = orig_clip(params, max_norm, *a, **k)
        norms.append(float(tn))
        return tn

    torch.nn.utils.clip_grad_norm_ = clip_wrap
    try:
        vl, al, ent = agent.update(st)
    finally:
        torch.nn.utils.clip_grad_norm_ = orig_clip
    pol.evaluate_actions = orig_eval
    rng_after_update = torch.get_rng_state()
    torch.set_rng_state(rng_before_update)
    perms = np.stack([torch.randperm(N * T).numpy() for _ in range(E)]).astype(np.int64)
    assert torch.equal(torch.get_rng_state(), rng_after_update)
    final = flat_params(pol)
    st.after_update()
    if not stride:
        save(fname, init_params=init, final_params=final, names=param_names(pol),
             obs_u8=obs_u8, exp_noise=np.stack(noise), values=np.stack(values),
             actions=np.stack(actions).astype(np.int64), action_log_probs=np.stack(logps),
             rewards=np.stack(rewards), masks=np.stack(masks), next_value=next_value.numpy(),
             returns=returns, value_preds_after=vpreds, perms=perms,
             mb0_values=mb_records[0]["values"], mb0_logp=mb_records[0]["logp"],
             mb_entropy=np.array([r["entropy"] for r in mb_records]),
             mb0_clipped_grad=grads[0], last_clipped_grad=grads[-1],
             losses=np.array([vl, al, ent]),
             meta=np.array([hidden, N, T, E, Mb]), lr=np.array([lr]))
        return
    extra = {}
    if obs_seed is not None:
        # the float64 gradient of the first minibatch (oracle/torch_ref: the same loss by
        # float64 autograd, on the reference's recorded rollout): at 16,384 samples a
        # weight gradient sums up to 6.5 M products, and the reference's own fp32
        # arithmetic is 1e-5 .. 3e-5 from float64 — the replay is held to its precision
        # against this (tests/helpers/gradcheck.py's rule), not to 1e-5 of the fp32 record
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
        from oracle import torch_ref as TR
        T_, N_ = T, N
        fl = lambda t: torch.as_tensor(t).reshape(T_ * N_)  # noqa: E731
        adv = torch.from_numpy(returns[:-1] - vpreds[:-1])
        adv = (adv - adv.mean()) / (adv.std() + 1e-5)   # ppo.py:35-37, fp32 as the reference
        p64 = TR.unflatten(torch.from_numpy(init), hidden, dtype=torch.float64, requires_grad=True)
        torch.set_num_threads(8)
        g64, _ = TR.minibatch_grads(p64, all_obs[:T].reshape(T * N, 4, 84, 84),
                                    torch.from_numpy(np.stack(actions).astype(np.int64)).reshape(-1),
                                    fl(np.stack(logps)), fl(adv), fl(vpreds[:-1]), fl(returns[:-1]),
                                    clip=0.1, value_coef=0.5, entropy_coef=0.001, chunk=1024)
        torch.set_num_threads(1)
        extra.update(digest("mb0_grad_f64", torch.cat([t.detach().reshape(-1) for t in g64]).numpy(), pol, stride))
    if obs_seed is None:
        extra["obs_u8"] = obs_u8
    else:
        import zlib
        extra["obs_seed"] = np.array([obs_seed])
        extra["obs_check"] = np.array([int(obs_u8.sum(dtype=np.int64)), zlib.crc32(obs_u8.tobytes())], np.int64)
    save(fname, init_params=init, rng_after_init=rng_init, names=param_names(pol),
         actions=np.stack(actions).astype(np.int64), action_log_probs=np.stack(logps), values=np.stack(values),
         rewards=np.stack(rewards), masks=np.stack(masks), returns=returns, perms=perms,
         mb_entropy=np.array([r["entropy"] for r in mb_records]), losses=np.array([vl, al, ent]),
         sampling_margin=np.array([margin]), total_norms=np.array(norms), exp_noise=np.stack(noise),
         value_preds_after=vpreds, next_value=next_value.numpy(),
         meta=np.array([hidden, N, T, E, Mb]), lr=np.array([lr]), **extra,
         **digest("final_params", final, pol, stride), **digest("mb0_preclip_grad", preclip[0], pol, stride))


# ---------------------------------------------------------------------------
# (6) GRU + vector obs evaluate_actions / act (T/ model.py:111-166,192-199)
# ---------------------------------------------------------------------------
def gen_gru(S, M, P):
    torch.manual_seed(11)
    hidden, V, N, T = 32, 14, 4, 8
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase,
                   base_kwargs={"recurrent": True, "hidden_size": hidden}, vector_obs_len=V)
    g = torch.Generator().manual_seed(5)
    obs_u8 = torch.randint(0, 256, (T, N, 4, 84, 84), dtype=torch.uint8, generator=g)
    vec = torch.rand(T, N, V, generator=g)
    masks = (torch.rand(T, N, 1, generator=g) > 0.25).float()
    masks[0] = 1.0
    h0 = torch.randn(N, hidden, generator=g)
    actions = torch.randint(0, 8, (T * N, 1), generator=g)
    with torch.no_grad():
        val, logp, ent, hT = pol.evaluate_actions((obs_u8.float() / 255.0).view(T * N, 4, 84, 84),
                                                  vec.view(T * N, V), h0, masks.view(T * N, 1), actions)
        # single-step act path (x.size(0) == hxs.size(0) branch)
        v1, f1, h1 = pol.base((obs_u8[0].float() / 255.0), vec[0], h0, masks[0])
    save("gru_eval.npz", params=flat_params(pol), names=param_names(pol),
         obs_u8=obs_u8.numpy(), vector_obs=vec.numpy(), masks=masks.numpy(), h0=h0.numpy(),
         actions=actions.numpy(), values=val.numpy(), log_probs=logp.numpy(),
         entropy=np.array([float(ent)]), hT=hT.numpy(), step_value=v1.numpy(),
         step_features=f1.numpy(), step_h=h1.numpy(), meta=np.array([hidden, V, N, T]))


# ---------------------------------------------------------------------------
# (6b) one whole recurrent iteration (T/ GRU + vector obs): rollout (act with the
#      hidden-state carry, masks with zeros), get_value, compute_returns, then the
#      reference's own PPO.update over recurrent_generator (storage.py:162-223,
#      model.py:111-166, algo/ppo.py:43-96): BPTT -> clip_grad_norm_ -> Adam
# ---------------------------------------------------------------------------
def gen_gru_update(S, M, P, *, hidden=32, V=14, N=8, T=16, E=2, Mb=2, lr=1e-3, fname="gru_update.npz", stride=0):
    torch.manual_seed(31)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase,
                   base_kwargs={"recurrent": True, "hidden_size": hidden}, vector_obs_len=V)
    # widen the action head and give the GRU non-zero biases so that the policy is
    # far from uniform (ratio clipping engages in epoch 2) — still the module's own forward
    gw = torch.Generator().manual_seed(32)
    with torch.no_grad():
        pol.dist.linear.weight.mul_(40.0)
        pol.base.gru.bias_ih_l0.copy_(torch.rand(3 * hidden, generator=gw) * 0.6 - 0.3)
        pol.base.gru.bias_hh_l0.copy_(torch.rand(3 * hidden, generator=gw) * 0.6 - 0.3)
    agent = P.PPO(pol, 0.1, E, Mb, 0.5, 0.01, lr=lr, eps=1e-5, max_grad_norm=0.5)
    st = S.RolloutStorage(T, N, (4, 84, 84), [V], Discrete(8), pol.recurrent_hidden_state_size)
    init = flat_params(pol)
    rng_init = torch.get_rng_state().numpy().copy()   # the default generator after construction
    genv = torch.Generator().manual_seed(321)

    def frame():   # 21x21 random bytes upsampled x4: full 0..255 range, compressible fixture
        lo = torch.randint(0, 256, (N, 4, 21, 21), dtype=torch.uint8, generator=genv)
        return lo.repeat_interleave(4, 2).repeat_interleave(4, 3).contiguous()

    obs_u8 = np.zeros((T + 1, N, 4, 84, 84), np.uint8)
    vec = np.zeros((T + 1, N, V), np.float32)
    o0 = frame()
    obs_u8[0] = o0.numpy()
    st.obs[0].copy_(o0.float() / 255.0)
    v0 = torch.rand(N, V, generator=genv)
    vec[0] = v0.numpy()
    st.vector_obs[0].copy_(v0)
    h0 = torch.randn(N, hidden, generator=genv) * 0.5        # a mid-training rollout's carried state
    st.recurrent_hidden_states[0].copy_(h0)
    m0 = (torch.rand(N, 1, generator=genv) > 0.3).float()     # episodes that ended on the previous step
    st.masks[0].copy_(m0)
    noise, values, actions, logps, rewards, masks = [], [], [], [], [], []
    for step in range(T):
        with torch.no_grad():
            rs = torch.get_rng_state()
            value, action, logp, hxs = pol.act(st.obs[step], st.vector_obs[step],
                                               st.recurrent_hidden_states[step], st.masks[step])
            after = torch.get_rng_state()
            torch.set_rng_state(rs)
            En = torch.empty(N, 8).exponential_(1)
            assert torch.equal(torch.get_rng_state(), after)
        o = frame()
        vo = torch.rand(N, V, generator=genv)
        rew = torch.rand(N, 1, generator=genv)
        done = torch.rand(N, generator=genv) < 0.25
        mk = torch.FloatTensor([[0.0] if d else [1.0] for d in done])
        bmk = torch.ones(N, 1)
        obs_u8[step + 1] = o.numpy()
        vec[step + 1] = vo.numpy()
        st.insert(o.float() / 255.0, vo, hxs, action, logp, value, rew, mk, bmk)
        noise.append(En.numpy()); values.append(value.numpy()); actions.append(action.numpy())
        logps.append(logp.numpy()); rewards.append(rew.numpy()); masks.append(mk.numpy())
    hid_T = st.recurrent_hidden_states[-1].numpy().copy()
    with torch.no_grad():
        next_value = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1],
                                   st.masks[-1]).detach()
    st.compute_returns(next_value, True, 0.99, 0.95, False)
    returns = st.returns.numpy().copy()
    vpreds = st.value_preds.numpy().copy()

    # capture: env orders (replayed randperms), per-minibatch losses (the .item()
    # calls of ppo.py:86-88, on graph tensors only), the pre-clip gradient and total
    # norm (clip_grad_norm_'s input and result), the clipped gradient (at step())
    rng_before_update = torch.get_rng_state()
    items, preclip, norms, clipped = [], [], [], []
    orig_item = torch.Tensor.item

    def item_wrap(self):
        v = orig_item(self)
        if self.requires_grad:
            items.append(v)
        return v

    orig_clip = torch.nn.utils.clip_grad_norm_

    def clip_wrap(params, max_norm, *a, **k):
        params = list(params)
        preclip.append(np.concatenate([p.grad.reshape(-1).numpy().copy() for p in params]))
        tn = orig_clip(params, max_norm, *a, **k)
        norms.append(float(tn))
        return tn

    orig_step = agent.optimizer.step

    def step_wrap(*a, **k):
        clipped.append(np.concatenate([p.grad.reshape(-1).numpy().copy() for p in pol.parameters()]))
        return orig_step(*a, **k)

    agent.optimizer.step = step_wrap
    torch.Tensor.item = item_wrap
    torch.nn.utils.clip_grad_norm_ = clip_wrap
    try:
        vl, al, ent = agent.update(st)
    finally:
        torch.Tensor.item = orig_item
        torch.nn.utils.clip_grad_norm_ = orig_clip
    rng_after_update = torch.get_rng_state()
    torch.set_rng_state(rng_before_update)
    perms = np.stack([torch.randperm(N).numpy() for _ in range(E)]).astype(np.int64)
    assert torch.equal(torch.get_rng_state(), rng_after_update)
    assert len(items) == 3 * E * Mb and len(preclip) == E * Mb == len(clipped)
    for g, c, tn in zip(preclip, clipped, norms):   # step() saw clip_grad_norm_'s scaling of its input
        np.testing.assert_allclose(c, g * min(0.5 / (tn + 1e-6), 1.0), rtol=1e-6, atol=1e-12)
    final = flat_params(pol)
    common = dict(init_params=init, rng_after_init=rng_init, names=param_names(pol),
                  obs_u8=obs_u8, vector_obs=vec, h0=h0.numpy(), masks0=m0.numpy(), hidden_T=hid_T,
                  values=np.stack(values), actions=np.stack(actions).astype(np.int64),
                  action_log_probs=np.stack(logps), rewards=np.stack(rewards), masks=np.stack(masks),
                  returns=returns, perms=perms, mb_losses=np.array(items, np.float64).reshape(E * Mb, 3),
                  total_norms=np.array(norms), losses=np.array([vl, al, ent]), exp_noise=np.stack(noise),
                  next_value=next_value.numpy(), value_preds_after=vpreds,
                  meta=np.array([hidden, V, N, T, E, Mb]), coefs=np.array([0.1, 0.5, 0.01]), lr=np.array([lr]))
    if stride:
        save(fname, **common, **digest("final_params", final, pol, stride),
             **digest("mb0_preclip_grad", preclip[0], pol, stride))
        return
    save(fname, **common, final_params=final, mb0_preclip_grad=preclip[0], last_preclip_grad=preclip[-1])


# ---------------------------------------------------------------------------
# (7) clip_grad_norm_ + Adam.step (ppo.py:82-84; torch 2.10 semantics)
# ---------------------------------------------------------------------------
def gen_adam():
    torch.manual_seed(21)
    shapes = [(32, 4, 8, 8), (32,), (64, 50), (1,)]
    params = [torch.nn.Parameter(torch.randn(s) * 0.1) for s in shapes]
    init = np.concatenate([p.detach().reshape(-1).numpy() for p in params])
    opt = torch.optim.Adam(params, lr=1e-3, eps=1e-5)
    grads, clipped, after, norms = [], [], [], []
    for k in range(4):
        g = [torch.randn(s) * (3.0 if k % 2 == 0 else 0.01) for s in shapes]
        for p, gi in zip(params, g):
            p.grad = gi.clone()
        grads.append(np.concatenate([x.reshape(-1).numpy() for x in g]))
        tn = torch.nn.utils.clip_grad_norm_(params, 0.5)
        norms.append(float(tn))
        clipped.append(np.concatenate([p.grad.reshape(-1).numpy().copy() for p in params]))
        opt.step()
        after.append(np.concatenate([p.detach().reshape(-1).numpy().copy() for p in params]))
    save("adam_clip.npz", init=init, grads=np.stack(grads), clipped=np.stack(clipped),
         after=np.stack(after), total_norms=np.array(norms),
         sizes=np.array([int(np.prod(s)) for s in shapes]), lr=np.array([1e-3]),
         eps=np.array([1e-5]), max_norm=np.array([0.5]))


# ---------------------------------------------------------------------------
# (8) MLPBase submodules (c1; model.py:202-234 — forward itself is broken,
#     so the submodules are driven directly)
# ---------------------------------------------------------------------------
def gen_mlp(M, D):
    torch.manual_seed(4)
    base = M.MLPBase(4, recurrent=False, hidden_size=64)
    head = D.Categorical(64, 2)
    x = torch.randn(8, 4)
    with torch.no_grad():
        value = base.critic_linear(base.critic(x))
        feat = base.actor(x)
        dist = head(feat)
    save("mlp.npz", base_params=flat_params(base), base_names=param_names(base),
         head_params=flat_params(head), x=x.numpy(), value=value.numpy(),
         actor_features=feat.numpy(), norm_logits=dist.logits.numpy(),
         entropy=dist.entropy().numpy())


def main():
    torch.set_num_threads(1)  # as T/run.py:55
    want = set(sys.argv[1:])
    on = lambda k: not want or k in want  # noqa: E731
    S, M, D, P = load_ref("B")
    if on("gae"):
        gen_gae(S)
    if on("advnorm"):
        gen_advnorm(S, P)
    if on("sampler"):
        gen_sampler(S)
    if on("categorical"):
        gen_categorical(D)
    if on("cnn_update"):
        gen_cnn_update(S, M, P, hidden=64, N=4, T=4, E=2, Mb=2, lr=1e-3, fname="cnn_update.npz")
    if on("cnn_update_h512"):   # the production hidden size (c3), VERDICT r05 item 6
        gen_cnn_update(S, M, P, hidden=512, N=4, T=4, E=2, Mb=2, lr=1e-3, fname="cnn_update_h512.npz",
                       lowres=True, stride=8)
    if on("cnn_update_wide"):   # c3's hidden size at a minibatch wide enough for the production fc tiles
        seed = int(os.environ.get("GOLDEN_WIDE_SEED", "2027"))   # chosen for its sampling margin (2.9e-4)
        gen_cnn_update(S, M, P, hidden=512, N=128, T=128, E=1, Mb=1, lr=1e-4,
                       fname=os.environ.get("GOLDEN_WIDE_NAME", "cnn_update_wide.npz"), stride=8, obs_seed=seed)
    if on("adam"):
        gen_adam()
    if on("mlp"):
        gen_mlp(M, D)
    S, M, D, P = load_ref("T")
    if on("gru"):
        gen_gru(S, M, P)
    if on("gru_update"):
        gen_gru_update(S, M, P)
    if on("gru_update_h256"):   # c5's hidden size: the persistent split-bf16 GRU kernels, VERDICT r05 item 6
        gen_gru_update(S, M, P, hidden=256, V=14, N=8, T=16, E=2, Mb=2, lr=1e-3, fname="gru_update_h256.npz",
                       stride=8)


if __name__ == "__main__":
    main()
