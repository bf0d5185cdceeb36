"""A one-rank gloo process group with the collectives forced on (so the
bucketed gradient all-reduce runs on device tensors, its fc + heads tail on a
side stream): (1) a started bucket is pending until allreduce_grads joins it, and
_dist.assert_no_pending refuses a persistent-GRU launch meanwhile; (2) a
recurrent (GRU) PPO update runs its minibatches with the buckets joined before
every persistent GRU launch (the assertion inside train_minibatch_rec passes)
and trains.  Prints one JSON line (tests/test_dist_gpu.py)."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    from a2c_ppo_acktr import _dist
    _dist.force_collectives(True)
    dev = torch.device("cuda", 0)
    out = {}
    g = torch.arange(100, dtype=torch.float32, device=dev)
    ok_start = _dist.start_bucket(g[60:])
    out["pending_after_start"] = _dist.pending_buckets()
    try:
        _dist.assert_no_pending("probe")
        out["refused"] = False
    except RuntimeError:
        out["refused"] = True
    _dist.allreduce_grads(g)
    out["pending_after_join"] = _dist.pending_buckets()
    _dist.assert_no_pending("probe")
    out["bucket_started"] = bool(ok_start)
    # a recurrent update with the forced collectives
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import SyntheticVecEnv
    torch.manual_seed(3)
    N, T, H, V = 16, 8, 64, 6
    env = SyntheticVecEnv(N, seed=5, p_done=0.1, device=dev)
    pol = M.Policy((4, 84, 84), env.action_space, base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": H},
                   vector_obs_len=V)
    pol.to(dev)
    agent = PPO(pol, 0.1, 2, 4, 0.5, 0.01, lr=1e-3, eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [V], env.action_space, pol.recurrent_hidden_state_size,
                        obs_dtype=torch.uint8, device=dev)
    env.reset_into(st.obs[0])
    vec = torch.rand(N, V, device=dev)
    st.vector_obs[0].copy_(vec)
    before = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    for step in range(T):
        v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step], st.masks[step])
        r, m, bm = env.step_into(st.obs[step + 1], a)
        st.insert(st.obs[step + 1], vec, h, a, lp, v, r, m, bm)
    nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
    st.compute_returns(nv, True, 0.99, 0.95, False)
    losses = agent.update(st)
    torch.cuda.synchronize()
    after = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    out["losses_finite"] = all(torch.isfinite(torch.tensor(losses)).tolist())
    out["moved"] = float((after - before).abs().max())
    out["pending_at_end"] = _dist.pending_buckets()
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
