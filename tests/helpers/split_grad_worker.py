"""One process of tests/test_gpu_parity.py::test_split_minibatch_gradient_equals_single_gpu
(SURVEY §8e(ii)): the same global minibatch either on one rank (world 1) or
split over two ranks that each own half of the env lanes (world 2, gloo
collectives on device tensors, both ranks on the one GPU).  Writes the averaged
flat gradient after the product's all-reduce, the losses and the advantage
statistics to an .npz."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

T, N_GLOBAL, H, A = 8, 32, 128, 8
G_SPLIT = 2   # the split the global minibatch is built for


class _GradCapture(object):
    """Stands in for FlatAdam at the end of a minibatch: runs the product's
    gradient all-reduce (_dist.allreduce_grads) and keeps Σg·(1/G)."""

    def _step_flat(self, eng):
        from a2c_ppo_acktr import _dist
        scale = _dist.allreduce_grads(eng.grad)
        self.grad = (eng.grad * scale).cpu().numpy()


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    dev = torch.device("cuda", 0)
    torch.manual_seed(7)
    pol = M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    with torch.no_grad():   # widen the heads so every loss branch carries weight
        pol.dist.linear.weight.mul_(30.0)
    pol.to(dev)
    eng = pol.hip_engine()
    # the global rollout, identical in every process
    g = torch.Generator().manual_seed(11)
    obs = torch.randint(0, 256, (T + 1, N_GLOBAL, 4, 84, 84), dtype=torch.uint8, generator=g)
    actions = torch.randint(0, A, (T, N_GLOBAL, 1), generator=g)
    logp = torch.log(torch.rand(T, N_GLOBAL, 1, generator=g)) * 0.3 - 2.0
    vpred = torch.randn(T + 1, N_GLOBAL, 1, generator=g) * 0.5
    rewards = torch.rand(T, N_GLOBAL, 1, generator=g)
    masks = (torch.rand(T + 1, N_GLOBAL, 1, generator=g) > 0.1).float()
    next_value = torch.randn(N_GLOBAL, 1, generator=g)
    # this process's lanes
    n = N_GLOBAL // world
    lanes = slice(rank * n, (rank + 1) * n)
    st = RolloutStorage(T, n, (4, 84, 84), [0], Discrete(A), 1, obs_dtype=torch.uint8, device=dev)
    st.obs.copy_(obs[:, lanes])
    st.actions.copy_(actions[:, lanes])
    st.action_log_probs.copy_(logp[:, lanes])
    st.value_preds.copy_(vpred[:, lanes])
    st.rewards.copy_(rewards[:, lanes])
    st.masks.copy_(masks[:, lanes])
    st.compute_returns(next_value[lanes].to(dev), True, 0.99, 0.95, False)
    adv = st.normalized_advantages()   # global statistics (3-double all-reduce at world 2)
    stats = st._adv_stats.cpu().numpy()
    # the global minibatch: B/2 local rows from each half of the lanes
    per = T * (N_GLOBAL // G_SPLIT) // 2
    rows = []
    for h in range(G_SPLIT):
        loc = torch.randperm(T * (N_GLOBAL // G_SPLIT), generator=torch.Generator().manual_seed(100 + h))[:per]
        rows.append(loc)
    if world == 1:
        nh = N_GLOBAL // G_SPLIT
        idx = torch.cat([(r // nh) * N_GLOBAL + h * nh + (r % nh) for h, r in enumerate(rows)])
    else:
        idx = rows[rank]
    hp = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.01, "use_clipped_value_loss": True}
    loss = torch.zeros(4, dtype=torch.float64, device=dev)
    cap = _GradCapture()
    eng.train_minibatch(st, adv, idx.to(dev), hp, loss, cap)
    from a2c_ppo_acktr import _dist
    _dist.allreduce_losses(loss)
    torch.cuda.synchronize()
    if rank == 0:
        np.savez(out, grad=cap.grad, loss=loss.cpu().numpy(), stats=stats)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
