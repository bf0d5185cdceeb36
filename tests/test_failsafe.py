"""Fail-safe update paths (GPU): a failure the reference would raise on, or a
persistent GRU kernel whose bounded wait runs out, must raise from PPO.update
*before* any optimizer step uses the bad data — parameters, Adam moments and
the step counter bit-unchanged — and a clean update must work right after.

Reference behaviour followed: the log_probs gather of an out-of-range stored
action raises inside evaluate_actions, before loss.backward() / optimizer.step()
(T/a2c_ppo_acktr/distributions.py:22, algo/ppo.py:57-84); the GRU forward of
model.py:116-165 cannot time out, so a timeout here is an error, never a result.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    from a2c_ppo_acktr import _hip
    return _hip


def _rollout(gpu, recurrent, N=64, T=16, H=64, V=14, seed=3):
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    torch.manual_seed(seed)
    V = V if recurrent else 0
    env = SyntheticVecEnv(N, seed=seed, p_done=0.05, device=gpu)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase,
                   base_kwargs={"recurrent": recurrent, "hidden_size": H}, vector_obs_len=V)
    pol.to(gpu)
    agent = PPO(pol, 0.1, 2, 2, 0.5, 0.001, lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [V], env.action_space, pol.recurrent_hidden_state_size,
                        obs_dtype=torch.uint8, device=gpu)
    env.reset_into(st.obs[0])

    def fill():
        for step in range(T):
            with torch.no_grad():
                v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                      st.masks[step])
            r, m, bm = env.step_into(st.obs[step + 1], a)
            st.insert(st.obs[step + 1], torch.rand(N, V, device=gpu) if V else st.vector_obs[step + 1], h, a, lp, v,
                      r, m, bm)
        with torch.no_grad():
            nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, False)
    return pol, agent, st, fill


def _state(pol, agent):
    eng = pol.hip_engine()
    opt = agent.optimizer
    return (eng.flat.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt.step_count)


def _assert_same(a, b):
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    assert a[3] == b[3]


def test_gru_timeout_raises_before_any_step(gpu):
    """Persistent GRU forward forced to give up its waits (bound 0 polls): the
    update raises RuntimeError, parameters / moments / step counter are
    bit-unchanged, and with the default bound the next update succeeds."""
    H_ = _hip()
    pol, agent, st, fill = _rollout(gpu, recurrent=True)
    assert H_.call("ppo_gru_persist_get") == 3
    fill()
    agent.update(st)            # a clean update first: Adam state exists
    st.after_update()
    fill()
    before = _state(pol, agent)
    H_.call("ppo_gru_persist_spin_set", 0)
    try:
        with pytest.raises(RuntimeError, match="timed out"):
            agent.update(st)
    finally:
        H_.call("ppo_gru_persist_spin_set", 1 << 21)
    torch.cuda.synchronize()
    _assert_same(_state(pol, agent), before)
    losses = agent.update(st)   # the same rollout, default bound: a normal step
    assert all(np.isfinite(losses))
    after = _state(pol, agent)
    assert after[3] == before[3] + 2 * 2
    assert (after[0] - before[0]).abs().max().item() > 0


def test_gru_timeout_in_evaluate_actions_raises(gpu):
    """evaluate_actions' multi-step branch (model.py:116-165) on the persistent
    kernel: a forced timeout raises instead of returning stale values."""
    H_ = _hip()
    pol, agent, st, fill = _rollout(gpu, recurrent=True, N=32, T=8)
    fill()
    T, N = 8, 32
    args = (st.obs[:-1].reshape(T * N, 4, 84, 84), st.vector_obs[:-1].reshape(T * N, -1),
            st.recurrent_hidden_states[0], st.masks[:-1].reshape(T * N, 1), st.actions.reshape(T * N, 1))
    with torch.no_grad():
        ok = pol.evaluate_actions(*args)
    H_.call("ppo_gru_persist_spin_set", 0)
    try:
        with pytest.raises(RuntimeError, match="timed out"):
            with torch.no_grad():
                pol.evaluate_actions(*args)
    finally:
        H_.call("ppo_gru_persist_spin_set", 1 << 21)
    with torch.no_grad():
        again = pol.evaluate_actions(*args)
    assert torch.equal(ok[0], again[0]) and torch.equal(ok[1], again[1])


@pytest.mark.parametrize("recurrent", [False, True])
def test_out_of_range_action_raises_before_any_step(gpu, recurrent):
    """Stored actions outside [0, A) in every lane of one step (so the update's
    first minibatch already holds one): IndexError with the true count (not
    multiplied by the epoch count), parameters / moments / step counter
    bit-unchanged; after the caller repairs the rollout, the update succeeds."""
    pol, agent, st, fill = _rollout(gpu, recurrent=recurrent)
    fill()
    agent.update(st)
    st.after_update()
    fill()
    before = _state(pol, agent)
    good = st.actions[3].clone()
    st.actions[3] = 99
    with pytest.raises(IndexError, match=r"\b64 stored action"):
        agent.update(st)
    torch.cuda.synchronize()
    _assert_same(_state(pol, agent), before)
    st.actions[3] = good
    losses = agent.update(st)
    assert all(np.isfinite(losses))
    assert _state(pol, agent)[3] == before[3] + 4


@pytest.mark.parametrize("recurrent", [False, True])
def test_out_of_range_action_mid_update(gpu, recurrent):
    """One bad stored action: as in the reference, the minibatches before the one
    holding it take their optimizer steps and the update raises there — the step
    counter advances by exactly that many steps (found by replaying the update's
    randperm draws on the default generator) and no later step lands."""
    pol, agent, st, fill = _rollout(gpu, recurrent=recurrent)
    fill()
    agent.update(st)
    st.after_update()
    fill()
    before = _state(pol, agent)
    N, T, E, M = 64, 16, 2, 2
    st.actions[3, 5] = 99
    rng = torch.get_rng_state()
    first = None
    for e in range(E):   # the update's sampler draws (storage.py:138-141 / :170)
        perm = torch.randperm(N if recurrent else N * T)
        per = (N if recurrent else N * T) // M
        for j in range(M):
            chunk = perm[j * per:(j + 1) * per]
            hit = (chunk == 5).any() if recurrent else (chunk == 3 * N + 5).any()
            if first is None and bool(hit):
                first = e * M + j
    torch.set_rng_state(rng)
    with pytest.raises(IndexError, match=r"\b1 stored action"):
        agent.update(st)
    torch.cuda.synchronize()
    after = _state(pol, agent)
    assert after[3] == before[3] + first
    if first == 0:
        _assert_same(after, before)
