"""Per-tensor gradient check against a float64 reference, with the torch fp32
autograd gradient of the same minibatch as the precision yardstick (shared by
test_full_size.py and test_half.py)."""
import numpy as np
import torch

from oracle import ppo_oracle as O


def check_grads(got_flat, ref_list, shapes, fp32_flat=None, fro_tol=3e-5, max_tol=1e-4, ratio=2.0, floor=1e-6):
    """Per tensor, against the float64 reference: relative Frobenius error
    ||err||/||ref|| <= fro_tol and max |err| <= max_tol * max|ref|; and, where the
    same gradient computed by torch's own fp32 autograd is given (fp32_flat: the
    reference's precision), our Frobenius error <= ratio x torch fp32's + floor
    (floor: 1e-6 relative, ~16 fp32 ulps — where torch's own error happens to be
    far below that, e.g. a bias summed over few terms, the ratio alone is noise);
    where torch fp32's own error exceeds fro_tol / max_tol, ratio x torch's error
    replaces them (the bar is the reference's own arithmetic).

    Why not 1e-5 of max|ref| element-wise at these sizes: a weight gradient here
    sums 16 k - 26 M products (conv1 at 65,536 rows: 26 M per element) and a few
    pre-activations / clip ratios sit within an fp32 rounding of a ReLU or clamp
    boundary, so every fp32 implementation lands 1e-5 .. 3e-5 from float64 —
    measured for torch fp32 autograd on the same minibatch (printed beside ours,
    e.g. conv1 weight at c3: torch 1.5e-5 max / 9.4e-6 Frobenius, ours 2.0e-5 /
    1.1e-5).  The bound that matters is the last one: no less accurate than the
    reference's own arithmetic."""
    got = O.unflatten(got_flat, shapes)
    f32 = O.unflatten(fp32_flat, shapes) if fp32_flat is not None else None
    bad = []
    for (name, _), ref in zip(shapes, ref_list):
        ref = ref.detach().cpu().numpy() if torch.is_tensor(ref) else ref
        scale, norm = max(np.abs(ref).max(), 1e-12), max(np.linalg.norm(ref), 1e-12)
        err = got[name] - ref
        mx, fro = np.abs(err).max() / scale, np.linalg.norm(err) / norm
        line = f"{name:28s} max|g| {scale:.3e}  HIP max {mx:.2e} fro {fro:.2e}"
        ok = fro <= fro_tol and mx <= max_tol
        if f32 is not None:
            e32 = f32[name] - ref
            mx32, fro32 = np.abs(e32).max() / scale, np.linalg.norm(e32) / norm
            line += f"  | torch-fp32 max {mx32:.2e} fro {fro32:.2e}"
            # where torch's own fp32 error exceeds the absolute bounds, the bound is
            # the reference's precision: within ratio x torch fp32 (+ floor)
            ok = (fro <= max(fro_tol, ratio * fro32) and mx <= max(max_tol, ratio * mx32)
                  and fro <= ratio * fro32 + floor)
        print(line, flush=True)
        if not ok:
            bad.append(line)
    assert not bad, bad
