"""Per-pixel error of ppo_conv2_fwd / _mask vs torch float64 (diagnostic for the
lone-pixel launch): prints the pixels whose error exceeds 1e-5 of max |ref|."""
import sys, torch, torch.nn.functional as F
sys.path.insert(0, "tests")
from test_gpu_parity import _hip, _packed, _s
Hh = _hip()
gpu = torch.device("cuda:0")
for B in (300, 4096):
    w, packed, pk = _packed(gpu, 64, 21)
    g = torch.Generator().manual_seed(22)
    a1 = torch.relu(torch.randn(B, 20, 20, 32, generator=g))
    b2 = torch.randn(64, generator=g) * 0.1
    a1_d, b2_d = a1.cuda(), b2.cuda()
    ref = torch.relu(F.conv2d(a1.double().permute(0, 3, 1, 2), w["w2"].double(), b2.double(), stride=2)).permute(0, 2, 3, 1)
    for name in ("ppo_conv2_fwd", "ppo_conv2_fwd_mask"):
        out = torch.full((B, 9, 9, 64), float("nan"), device=gpu)
        bits = torch.zeros(B * 81, dtype=torch.int64, device=gpu)
        if name == "ppo_conv2_fwd":
            Hh.call(name, a1_d.data_ptr(), B, pk[0], b2_d.data_ptr(), out.data_ptr(), _s())
        else:
            Hh.call(name, a1_d.data_ptr(), B, pk[0], b2_d.data_ptr(), out.data_ptr(), bits.data_ptr(), _s())
        torch.cuda.synchronize()
        e = (out.cpu().double() - ref).abs()
        tol = 1e-5 * ref.abs().max().item()
        bad = (e > tol) | torch.isnan(e)
        pix = bad.any(3).any(0).nonzero().tolist()
        imgs = bad.any(3).any(2).any(1).nonzero().flatten().tolist()
        print(B, name, "bad pixels", pix[:10], "n imgs", len(imgs), imgs[:8], "max err", e.nan_to_num(1e9).max().item(), flush=True)
