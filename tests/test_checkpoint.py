"""Checkpoints (reference T/run.py:251-262 save, :64-71 load):
state_dict files that load with weights_only=True round-trip the policy, ob_rms
and the Adam state bit for bit, and a run resumed from one continues exactly
like the uninterrupted run (GPU test)."""
import numpy as np
import pytest
import torch

from a2c_ppo_acktr import checkpoint as C
from a2c_ppo_acktr import model as M
from a2c_ppo_acktr.algo import PPO
from a2c_ppo_acktr.synthetic import Discrete


def _policy(H=64, recurrent=False, V=0, seed=3):
    torch.manual_seed(seed)
    return M.Policy((4, 84, 84), Discrete(6), base=M.CNNBase, base_kwargs={"recurrent": recurrent, "hidden_size": H},
                    vector_obs_len=V)


@pytest.mark.parametrize("recurrent,V", [(False, 0), (True, 14)])
def test_roundtrip_cpu(tmp_path, recurrent, V):
    pol = _policy(recurrent=recurrent, V=V)
    agent = PPO(pol, 0.1, 2, 2, 0.5, 0.01, lr=3e-4, eps=1e-5, max_grad_norm=0.5)
    n = sum(p.numel() for p in pol.parameters())
    g = torch.Generator().manual_seed(0)
    agent.optimizer.load_state_dict({"step": 7, "exp_avg": torch.randn(n, generator=g),
                                     "exp_avg_sq": torch.rand(n, generator=g),
                                     "param_groups": [{"lr": 1.25e-4, "betas": (0.9, 0.999), "eps": 1e-5,
                                                       "weight_decay": 0, "amsgrad": False}]})
    ob_rms = C.RunningMeanStd(np.arange(12, dtype=np.float64).reshape(3, 4), np.ones((3, 4)), 17.0)
    path = str(tmp_path / "ck" / "ObtRetro-v6.pt")
    C.save_checkpoint(path, pol, ob_rms, agent=agent, extra={"update": 3})
    # a plain-tensor file: the safe loader accepts it
    raw = torch.load(path, weights_only=True)
    assert raw["format"] == C.FORMAT and raw["extra"] == {"update": 3}
    torch.manual_seed(99)   # the rebuilt policy draws different initial weights, then loads
    agent2_pol = _policy(recurrent=recurrent, V=V, seed=99)
    agent2 = PPO(agent2_pol, 0.1, 2, 2, 0.5, 0.01, lr=1.0, eps=1e-5, max_grad_norm=0.5)
    pol2, ob2 = C.load_checkpoint(path, actor_critic=agent2_pol, agent=agent2)
    for (k, a), (k2, b) in zip(pol.state_dict().items(), pol2.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    assert np.array_equal(ob2.mean, ob_rms.mean) and ob2.count == 17.0
    o1, o2 = agent.optimizer.state_dict(), agent2.optimizer.state_dict()
    assert o2["step"] == 7 and torch.equal(o1["exp_avg"], o2["exp_avg"]) and torch.equal(o1["exp_avg_sq"],
                                                                                        o2["exp_avg_sq"])
    assert agent2.optimizer.param_groups[0]["lr"] == 1.25e-4
    # rebuilt from the recorded constructor config
    pol3, _ = C.load_checkpoint(path)
    assert pol3.is_recurrent == recurrent and type(pol3.base) is M.CNNBase
    assert pol3.dist.linear.weight.shape == (6, 64)
    for a, b in zip(pol.parameters(), pol3.parameters()):
        assert torch.equal(a, b)


def test_reference_pickle_form_still_works(tmp_path):
    """T/run.py:259-262 pickles [actor_critic, ob_rms]; our Policy pickles (no engine
    state).  Loading it back needs weights_only=False — acceptable for a file this
    test wrote itself, never for a reference artefact."""
    pol = _policy()
    path = str(tmp_path / "legacy.pt")
    torch.save([pol, None], path)
    pol2, ob = torch.load(path, weights_only=False)
    assert ob is None
    for a, b in zip(pol.parameters(), pol2.parameters()):
        assert torch.equal(a, b)


def test_mismatched_checkpoint_raises(tmp_path):
    path = str(tmp_path / "a.pt")
    C.save_checkpoint(path, _policy(H=64))
    with pytest.raises((KeyError, ValueError)):
        C.load_checkpoint(path, actor_critic=_policy(H=128))
    torch.save({"format": "other"}, path)
    with pytest.raises(ValueError):
        C.load_checkpoint(path)


@pytest.mark.gpu
def test_resume_is_bit_identical(gpu, tmp_path):
    """Train one update, checkpoint, then apply a second update both with the live
    objects and with objects restored from the file (same rollouts, same host RNG
    state for the minibatch permutations): parameters and losses are identical."""
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv

    N, T = 8, 16
    pol = _policy().to(gpu)
    agent = PPO(pol, 0.1, 2, 2, 0.5, 0.01, lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(6), 1, obs_dtype=torch.uint8, device=gpu)
    env = SyntheticVecEnv(N, num_actions=6, seed=5, p_done=0.2, device=gpu)
    env.reset_into(st.obs[0])

    def rollout(policy):
        for step in range(T):
            v, a, lp, h = policy.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                     st.masks[step])
            r, m, bm = env.step_into(st.obs[step + 1], a)
            st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, r, m, bm)
        nv = policy.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, False)

    rollout(pol)
    agent.update(st)
    st.after_update()
    path = str(tmp_path / "ck.pt")
    C.save_checkpoint(path, pol, None, agent=agent)
    rollout(pol)
    rng = torch.get_rng_state()
    l1 = agent.update(st)
    p1 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu()
    pol2 = _policy(seed=77).to(gpu)   # (re-seeds the global generator)
    agent2 = PPO(pol2, 0.1, 2, 2, 0.5, 0.01, lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    C.load_checkpoint(path, device=gpu, actor_critic=pol2, agent=agent2)
    torch.set_rng_state(rng)   # same minibatch permutations as the live run
    l2 = agent2.update(st)
    p2 = torch.cat([p.detach().reshape(-1) for p in pol2.parameters()]).cpu()
    assert l1 == l2
    assert torch.equal(p1, p2)
