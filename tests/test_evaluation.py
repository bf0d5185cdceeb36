"""Evaluation path (SURVEY §8f row f4, T/run_evaluation.py:25-122): batch-1
deterministic acting with the GRU state carried across steps, replayed from a
HIP graph — bit-identical to eager Policy.act step by step, and to the oracle's
float64 forward within fp32 tolerance."""
import numpy as np
import pytest
import torch

from a2c_ppo_acktr import model as M
from a2c_ppo_acktr.synthetic import Discrete

pytestmark = pytest.mark.gpu


def _policy(recurrent, H, V, seed=4):
    torch.manual_seed(seed)
    return M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": recurrent, "hidden_size": H},
                    vector_obs_len=V)


@pytest.mark.parametrize("recurrent,H,V", [(True, 256, 14), (False, 512, 0)])
def test_graphed_actor_matches_eager(gpu, recurrent, H, V):
    from a2c_ppo_acktr.evaluation import GraphedActor
    pol = _policy(recurrent, H, V).to(gpu)
    ga = GraphedActor(pol, num_envs=1)
    g = torch.Generator().manual_seed(9)
    hx_e = torch.zeros(1, pol.recurrent_hidden_state_size)      # host tensors, as run_evaluation.py keeps them
    hx_g = hx_e.clone()
    masks = torch.zeros(1, 1)
    for step in range(6):
        obs = torch.rand(1, 4, 84, 84, generator=g).to(gpu)
        vec = torch.rand(1, V, generator=g).to(gpu)
        with torch.no_grad():
            ve, ae, le, hx_e = pol.act(obs, vec, hx_e, masks, deterministic=True)
        vg, ag, lg, hx_g = ga.act(obs, vec, hx_g, masks)
        for a, b in ((ve, vg), (ae, ag), (le, lg), (hx_e, hx_g)):
            assert torch.equal(a.to(gpu), b.to(gpu)), step
        masks.fill_(0.0 if step == 3 else 1.0)   # an episode end resets the GRU state
        if step == 2:   # parameters trained in place between steps: the graph follows
            with torch.no_grad():
                for p in pol.parameters():
                    p.mul_(1.01)


def test_graphed_actor_vs_oracle(gpu):
    from a2c_ppo_acktr.evaluation import GraphedActor
    from oracle import ppo_oracle as O
    H, V = 256, 14
    pol = _policy(True, H, V)
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy().astype(np.float64)
    p = O.unflatten(flat, O.cnn_param_shapes(H, recurrent=True, vector_obs_len=V))
    pol.to(gpu)
    ga = GraphedActor(pol)
    g = torch.Generator().manual_seed(1)
    obs = torch.rand(1, 4, 84, 84, generator=g)
    vec = torch.rand(1, V, generator=g)
    h0 = torch.rand(1, H, generator=g)
    v, a, lp, h1 = ga.act(obs.to(gpu), vec.to(gpu), h0.to(gpu), torch.ones(1, 1, device=gpu))
    out = O.recurrent_forward(p, obs.numpy().astype(np.float64), vec.numpy().astype(np.float64),
                              h0.numpy().astype(np.float64), np.ones((1, 1)))
    value, logits, hT = out[0], out[1], out[2]["out"]
    np.testing.assert_allclose(v.cpu().numpy().ravel(), np.ravel(value), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(h1.cpu().numpy(), np.reshape(hT, (1, H)), rtol=1e-4, atol=1e-5)
    assert int(a.item()) == int(np.argmax(logits.ravel()))


def test_graphed_replay_carries_hidden_state(gpu):
    """GraphedActor.replay (the evaluation loop's fast path: inputs written in place
    into ga.obs / ga.vec / ga.masks, the new hidden state fed back inside the
    graph) equals eager Policy.act step by step over a masked sequence, bit for bit."""
    from a2c_ppo_acktr.evaluation import GraphedActor
    H, V = 256, 14
    pol = _policy(True, H, V).to(gpu)
    ga = GraphedActor(pol, carry_hidden=True)
    g = torch.Generator().manual_seed(5)
    hx = torch.zeros(1, H, device=gpu)
    for step in range(8):
        obs = torch.rand(1, 4, 84, 84, generator=g).to(gpu)
        vec = torch.rand(1, V, generator=g).to(gpu)
        m = torch.full((1, 1), 0.0 if step == 4 else 1.0, device=gpu)
        with torch.no_grad():
            ve, ae, le, hx = pol.act(obs, vec, hx, m, deterministic=True)
        ga.obs.copy_(obs)
        ga.vec.copy_(vec)
        ga.masks.copy_(m)
        vg, ag, lg, hg = ga.replay()
        for a, b in ((ve, vg), (ae, ag), (le, lg), (hx, hg), (hx, ga.hxs)):
            assert torch.equal(a, b), step


def test_graphed_actor_recaptures_on_precision_change(gpu):
    """Policy.half() / float() after a GraphedActor was built: the next act follows
    the new arithmetic mode (re-captured), i.e. equals eager acting in that mode."""
    from a2c_ppo_acktr.evaluation import GraphedActor
    pol = _policy(False, 512, 0).to(gpu)
    ga = GraphedActor(pol)
    obs = torch.rand(1, 4, 84, 84, generator=torch.Generator().manual_seed(2)).to(gpu)
    hx, m = torch.zeros(1, 1, device=gpu), torch.ones(1, 1, device=gpu)
    n0 = ga.captures
    for mode in ("half", "float"):
        getattr(pol, mode)()
        with torch.no_grad():
            ve = pol.act(obs, None, hx, m, deterministic=True)[0].clone()
        vg = ga.act(obs, None, hx, m)[0]
        assert torch.equal(ve, vg), mode
    assert ga.captures == n0 + 2
