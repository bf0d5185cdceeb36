"""RCCL on the hardware at hand (the reference pattern replaced is the
flat-gradient Allreduce / size of large-scale-curiosity/mpi_utils.py:27-28):
every collective of the multi-GPU protocol (_dist.py: parameter broadcast,
advantage-statistics all-reduce, per-minibatch flat-gradient all-reduce, loss
all-reduce) forced through a one-rank RCCL communicator, interleaved with the
engine's raw-stream launches.  A one-rank sum is exact, so one c3 iteration
must give bit-identical parameters, Adam moments and losses with and without
the collectives — which fails if RCCL ran out of stream order with the kernels
that produce or consume the gradient (the fc + heads bucket is reduced on a side
stream while the conv backward runs, _dist.start_bucket)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_forced_rccl_iteration_bit_identical(tmp_path, gpu):
    worker = os.path.join(os.path.dirname(__file__), "helpers", "rccl_worker.py")
    outs = []
    for force in (0, 1):
        out = str(tmp_path / f"r{force}.npz")
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        r = subprocess.run([sys.executable, worker, str(force), out], env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(np.load(out))
    a, b = outs
    # two per minibatch: the fc + heads bucket on the side stream, then the conv head
    assert a["allreduces"].size == 0 and b["allreduces"].size == 2 * 3 * 8
    for k in ("flat", "m", "v", "losses"):
        assert np.array_equal(a[k], b[k]), (k, np.abs(a[k] - b[k]).max())
    print("per-minibatch RCCL all-reduce ms:", np.round(b["allreduces"], 4).tolist())
