"""API robustness (round-1 advisor findings): a graphed actor survives eager acting
at other batch sizes and parameter re-binding, a checkpoint loaded through the
documented `load_checkpoint(path, device, agent=agent)` form trains the policy it
returned, restored Adam moments survive a device move, and stored actions outside
[0, A) raise as the reference's log_probs gather does (distributions.py:22)."""
import numpy as np
import pytest
import torch

from a2c_ppo_acktr import checkpoint as C
from a2c_ppo_acktr import model as M
from a2c_ppo_acktr.algo import PPO
from a2c_ppo_acktr.synthetic import Discrete


def _policy(H=64, recurrent=False, V=0, seed=3, A=6):
    torch.manual_seed(seed)
    return M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": recurrent, "hidden_size": H},
                    vector_obs_len=V)


def test_documented_load_form_binds_agent_policy(tmp_path):
    """load_checkpoint(path, agent=agent) loads into agent.actor_critic (the policy
    agent.update trains), not into a fresh Policy."""
    pol = _policy(seed=3)
    agent = PPO(pol, 0.1, 2, 2, 0.5, 0.01, lr=3e-4, eps=1e-5, max_grad_norm=0.5)
    path = str(tmp_path / "ck.pt")
    C.save_checkpoint(path, pol, None, agent=agent)
    pol2 = _policy(seed=11)
    agent2 = PPO(pol2, 0.1, 2, 2, 0.5, 0.01, lr=3e-4, eps=1e-5, max_grad_norm=0.5)
    got, _ = C.load_checkpoint(path, agent=agent2)
    assert got is agent2.actor_critic is pol2
    for a, b in zip(pol.parameters(), pol2.parameters()):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("recurrent,H,V", [(True, 256, 14), (False, 512, 0)])
def test_graphed_actor_survives_eager_batches_and_rebinding(gpu, recurrent, H, V):
    from a2c_ppo_acktr.evaluation import GraphedActor
    pol = _policy(H=H, recurrent=recurrent, V=V, A=8).to(gpu)
    ga = GraphedActor(pol, num_envs=1)
    g = torch.Generator().manual_seed(2)
    Hh = pol.recurrent_hidden_state_size

    def check(tag):
        obs = torch.rand(1, 4, 84, 84, generator=g).to(gpu)
        vec = torch.rand(1, V, generator=g).to(gpu)
        hx = torch.rand(1, Hh, generator=g).to(gpu)
        m = torch.ones(1, 1, device=gpu)
        with torch.no_grad():
            ve, ae, le, he = pol.act(obs, vec, hx, m, deterministic=True)
        vg, ag, lg, hg = ga.act(obs, vec, hx, m)
        for a, b in ((ve, vg), (ae, ag), (le, lg), (he, hg)):
            assert torch.equal(a, b), tag

    check("fresh")
    # an eager rollout at 64 envs grows (reallocates) the eager act workspace
    n = 64
    with torch.no_grad():
        pol.act(torch.rand(n, 4, 84, 84, device=gpu), torch.rand(n, V, device=gpu), torch.zeros(n, Hh, device=gpu),
                torch.ones(n, 1, device=gpu))
    torch.cuda.synchronize()
    check("after a 64-env eager act")
    captures = ga.captures
    # replacing the parameter storage re-binds the engine's flat buffer: re-capture
    with torch.no_grad():
        for p in pol.parameters():
            p.data = p.data.clone() * 1.01
    check("after re-binding")
    assert ga.captures == captures + 1


@pytest.mark.gpu
def test_restored_adam_moments_follow_device_move(gpu, tmp_path):
    """Moments restored on the host keep their values (and the step count's bias
    correction) when the first step runs on the GPU."""
    pol = _policy(H=64)
    agent = PPO(pol, 0.1, 1, 1, 0.5, 0.01, lr=1e-3, eps=1e-5, max_grad_norm=None)
    n = sum(p.numel() for p in pol.parameters())
    g = torch.Generator().manual_seed(4)
    m0, v0 = torch.randn(n, generator=g) * 1e-3, torch.rand(n, generator=g) * 1e-5
    agent.optimizer.load_state_dict({"step": 5, "exp_avg": m0.clone(), "exp_avg_sq": v0.clone(),
                                     "param_groups": [{"lr": 1e-3, "betas": (0.9, 0.999), "eps": 1e-5,
                                                       "weight_decay": 0, "amsgrad": False}]})
    p0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).double()
    pol.to(gpu)
    eng = pol.hip_engine()
    grad = torch.randn(n, generator=g) * 1e-2
    eng.grad.copy_(grad.to(gpu))
    agent.optimizer._step_flat(eng)
    torch.cuda.synchronize()
    # torch 2.10 Adam from the restored moments, step 6
    k, b1, b2, lr, eps = 6, 0.9, 0.999, 1e-3, 1e-5
    gd = grad.double()
    m = m0.double() * b1 + (1 - b1) * gd
    v = v0.double() * b2 + (1 - b2) * gd * gd
    ref = p0 - (lr / (1 - b1 ** k)) * m / (v.sqrt() / np.sqrt(1 - b2 ** k) + eps)
    got = eng.flat.cpu().double()
    assert torch.allclose(got, ref, rtol=0, atol=2e-6), (got - ref).abs().max()
    assert agent.optimizer.step_count == 6


@pytest.mark.gpu
def test_out_of_range_action_raises(gpu):
    from a2c_ppo_acktr.storage import RolloutStorage
    pol = _policy(H=64, A=6).to(gpu)
    agent = PPO(pol, 0.1, 1, 2, 0.5, 0.01, lr=1e-4, eps=1e-5, max_grad_norm=0.5)
    T, N = 4, 8
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(6), 1, obs_dtype=torch.uint8, device=gpu)
    st.actions.fill_(2)
    st.actions[1, 3] = 6          # outside [0, 6)
    st.compute_returns(torch.zeros(N, 1, device=gpu), True, 0.99, 0.95, False)
    with pytest.raises(IndexError):
        agent.update(st)
    # evaluate_actions marks such a row with a NaN log-prob
    obs = torch.zeros(2, 4, 84, 84, dtype=torch.uint8, device=gpu)
    _, lp, _, _ = pol.evaluate_actions(obs, None, None, None, torch.tensor([[1], [7]], device=gpu))
    lp = lp.cpu()
    assert torch.isfinite(lp[0]).all() and torch.isnan(lp[1]).all()
