"""One rank of the 2-process PPO tests on a single GPU: gloo collectives on
device tensors, each rank with its own env lanes.  Modes (argv[4]):
  update  (tests/test_gpu_parity.py::test_two_rank_update_one_gpu) a full update;
          prints the flat parameters' digest and the losses
  bucket  (tests/test_dist_gpu.py) one minibatch twice from the same parameters:
          first with the gradient collectives switched off (this rank's own
          gradient), then through the engine's bucketed path (fc + heads tail on
          the side stream during the conv backward, then the head); prints whether
          the reduced gradient equals (g_0 + g_1) / 2 bit for bit
  guard   (tests/test_dist_gpu.py) rank 1 alone stores an out-of-range action:
          every rank must skip every step (parameters, Adam moments, step count
          unchanged) and raise"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    mode = sys.argv[4] if len(sys.argv) > 4 else "update"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    dev = torch.device("cuda", 0)
    torch.manual_seed(1 + 100 * rank)   # different init per rank: PPO must broadcast rank 0's
    N, T, H = 8, 8, 64
    env = SyntheticVecEnv(N, seed=50 + rank, p_done=0.1, device=dev)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    pol.to(dev)
    if mode == "bucket":   # one minibatch, lr 0 (parameters stay), no clipping (coefficient 1)
        agent = PPO(pol, 0.1, 1, 1, 0.5, 0.01, lr=0.0, eps=1e-5, max_grad_norm=None)
    else:
        agent = PPO(pol, 0.1, 2, 2, 0.5, 0.01, lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [0], env.action_space, 1, obs_dtype=torch.uint8, device=dev)
    env.reset_into(st.obs[0])
    init = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    for step in range(T):
        v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step], st.masks[step])
        r, m, bm = env.step_into(st.obs[step + 1], a)
        st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, r, m, bm)
    nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
    st.compute_returns(nv, True, 0.99, 0.95, False)
    if mode == "bucket":
        return bucket(rank, world, pol, agent, st)
    if mode == "guard":
        return guard(rank, world, pol, agent, st, env.action_space.n)
    losses = agent.update(st)
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu()
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    same = all(torch.equal(gathered[0], g) for g in gathered)
    moved = float((flat - init.cpu()).abs().max())
    print(json.dumps({"rank": rank, "same": same, "moved": moved, "losses": list(losses),
                      "sum": float(flat.double().sum())}), flush=True)
    dist.destroy_process_group()


def bucket(rank, world, pol, agent, st):
    from a2c_ppo_acktr import _dist
    eng = pol.hip_engine()
    real = _dist.allreduce_grads, _dist.start_bucket
    _dist.allreduce_grads, _dist.start_bucket = (lambda g: 1.0), (lambda t: False)
    try:
        torch.manual_seed(7)              # the same minibatch draw in both passes
        agent.update(st)
        torch.cuda.synchronize()
        g_local = eng.grad.clone().cpu()
    finally:
        _dist.allreduce_grads, _dist.start_bucket = real
    flat0 = eng.flat.clone()
    torch.manual_seed(7)
    agent.update(st)
    torch.cuda.synchronize()
    g_red = eng.grad.cpu()                # clip + Adam leave Σ g / G there (coefficient 1)
    parts = [torch.empty_like(g_local) for _ in range(world)]
    dist.all_gather(parts, g_local)
    expect = parts[0]
    for p in parts[1:]:
        expect = expect + p
    expect = expect * (1.0 / world)
    print(json.dumps({"rank": rank, "equal": bool(torch.equal(g_red, expect)),
                      "maxdiff": float((g_red - expect).abs().max()),
                      "differ": bool(not torch.equal(parts[0], parts[1])),
                      "params_kept": bool(torch.equal(flat0, eng.flat)),
                      "tail_started": int(_dist._OVERLAP["on"])}), flush=True)
    dist.destroy_process_group()


def guard(rank, world, pol, agent, st, A):
    eng = pol.hip_engine()
    if rank == 1:
        st.actions[0, 0] = A + 3          # invalid on this rank only
    flat0 = eng.flat.clone()
    try:
        agent.update(st)
        raised = False
    except IndexError:
        raised = True
    torch.cuda.synchronize()
    opt = agent.optimizer
    moments_zero = opt.exp_avg is None or (not opt.exp_avg.any().item() and not opt.exp_avg_sq.any().item())
    print(json.dumps({"rank": rank, "raised": raised, "params_kept": bool(torch.equal(flat0, eng.flat)),
                      "moments_zero": bool(moments_zero), "step_count": opt.step_count}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
