"""Does a half-mode minibatch leave state that changes the next fp32 minibatch?
(fresh policy fp32 grad vs half-then-fp32 grad on identical inputs)"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ppo-dash_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import test_half as TH  # noqa: E402
from a2c_ppo_acktr import model as M  # noqa: E402
from a2c_ppo_acktr.synthetic import Discrete  # noqa: E402

gpu = torch.device("cuda:0")


def run(half_first):
    H, T, N, A = 512, 16, 256, 8
    torch.manual_seed(4)
    pol = M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    with torch.no_grad():
        pol.dist.linear.weight.mul_(30.0)
    pol.to(gpu)
    st = TH._storage(gpu, T, N, A, 5, torch.uint8)
    adv = torch.randn(T, N, generator=torch.Generator().manual_seed(6)).to(gpu)
    idx = torch.randperm(T * N, generator=torch.Generator().manual_seed(7))[:4096].to(gpu)
    eng = pol.hip_engine()
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)
    if half_first:
        pol.half()
        cap = TH._GradCapture()
        eng.train_minibatch(st, adv, idx, TH.HP, loss, cap)
        pol.float()
    cap = TH._GradCapture()
    eng.train_minibatch(st, adv, idx, TH.HP, loss, cap)
    torch.cuda.synchronize()
    return cap.grad.cpu()


g1, g2 = run(False), run(True)
d = (g1 - g2).abs()
print("bit-identical:", torch.equal(g1, g2), "max|diff|", d.max().item(), "max|g|", g1.abs().max().item())

# cross-process / garbage-memory sensitivity: poison the caching allocator's
# free memory with NaN, then recompute (uninitialised reads would show up)
junk = torch.full((1 << 28,), float("nan"), device=gpu)
del junk
g3 = run(False)
print("after NaN poison: bit-identical:", torch.equal(g1, g3), "nan:", torch.isnan(g3).any().item(),
      "checksum", float(g1.double().sum()), float(g3.double().sum()))
