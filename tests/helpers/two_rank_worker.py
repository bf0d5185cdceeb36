"""One rank of the 2-process PPO test on a single GPU (tests/test_gpu_parity.py::
test_two_rank_update_one_gpu): gloo collectives on device tensors, each rank
with its own env lanes; prints the flat parameters' digest and the losses."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
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


if __name__ == "__main__":
    main()
