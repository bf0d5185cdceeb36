"""One process of tests/test_rccl.py: one c3 iteration (CNNBase H=512, 4096
lanes x 128 steps, PPO 3 x 8; T/run.py:168-248 order) with or without every
collective running through a one-rank RCCL communicator (bench.py
--force-collectives).  Writes the flat parameters, Adam moments and losses."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    force, out = int(sys.argv[1]), sys.argv[2]
    N, T = int(os.environ.get("RCCL_N", "4096")), int(os.environ.get("RCCL_T", "128"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from a2c_ppo_acktr import _dist
    if force:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", device_id=dev)   # RCCL
        _dist.force_collectives(True)
        assert _dist.active()
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.model import CNNBase, Policy
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    torch.manual_seed(1)
    env = SyntheticVecEnv(N, seed=123, p_done=0.01, device=dev)
    pol = Policy((4, 84, 84), env.action_space, base=CNNBase, base_kwargs={"recurrent": False, "hidden_size": 512})
    pol.to(dev)
    agent = PPO(pol, 0.1, 3, 8, 0.5, 0.001, lr=1e-4, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [0], env.action_space, 1, obs_dtype=torch.uint8, device=dev)
    env.reset_into(st.obs[0])
    _dist.time_grads(True)
    for step in range(T):
        with torch.no_grad():
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step], st.masks[step])
        slot = st.obs[step + 1]
        r, m, bm = env.step_into(slot, a)
        st.insert(slot, st.vector_obs[step + 1], h, a, lp, v, r, m, bm)
    with torch.no_grad():
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
    st.compute_returns(nv, True, 0.99, 0.95, False)
    losses = agent.update(st)
    st.after_update()
    torch.cuda.synchronize()
    times = _dist.grad_allreduce_times()
    eng = pol.hip_engine()
    np.savez(out, flat=eng.flat.cpu().numpy(), m=agent.optimizer.exp_avg.cpu().numpy(),
             v=agent.optimizer.exp_avg_sq.cpu().numpy(), losses=np.array(losses),
             allreduces=np.array([t for t, _ in times]))
    if force:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
