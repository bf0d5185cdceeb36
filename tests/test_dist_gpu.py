"""The G>1 protocol on the device, with real sums over two ranks (two processes
sharing the one GPU, gloo collectives on device tensors; RCCL takes the same
calls on an 8-GPU node).  Complements tests/test_rccl.py, whose one-rank
communicator cannot tell a misordered reduce from a correct one (a one-rank sum
is the identity).

* the bucketed gradient all-reduce (`_dist.start_bucket`: the fc + heads tail
  reduced on a side stream while the conv backward runs, then the conv head on
  the current stream) gives exactly (g_0 + g_1) / 2 of the two ranks' own
  minibatch gradients;
* the optimizer-step guard is global: when ONE rank stores an out-of-range
  action, every rank skips every step of the update (parameters, Adam moments
  and step count unchanged on all ranks) and every rank raises, as a single
  process does (reference: the log_probs gather of distributions.py:22 raises
  before its optimizer step)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

WORKER = os.path.join(os.path.dirname(__file__), "helpers", "two_rank_worker.py")


def _run(mode):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), "2", port, mode], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e[-2000:]
        outs.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    return outs


def test_bucketed_allreduce_sums_two_ranks():
    outs = _run("bucket")
    for o in outs:
        assert o["differ"], "the two ranks' gradients must differ for the check to mean anything"
        assert o["tail_started"]
        assert o["equal"], o
        assert o["params_kept"]


def test_guard_skips_on_every_rank():
    outs = _run("guard")
    for o in outs:
        assert o["raised"], o
        assert o["params_kept"] and o["moments_zero"] and o["step_count"] == 0, o


def test_gru_launch_after_bucket_join():
    """Persistent GRU launches need their blocks co-resident; a collective kernel on
    the side stream could hold CUs they wait for.  A started gradient bucket is
    pending until allreduce_grads joins it (the current stream waits for it) and
    _dist.assert_no_pending refuses a persistent launch meanwhile; a recurrent
    update with the collectives forced on (one-rank gloo group on the device) runs
    every minibatch's GRU launches with no bucket pending, and trains."""
    import subprocess
    worker = os.path.join(os.path.dirname(__file__), "helpers", "rank1_gru_worker.py")
    r = subprocess.run([sys.executable, worker], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    o = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert o["bucket_started"] and o["pending_after_start"] == 1 and o["refused"]
    assert o["pending_after_join"] == 0 and o["pending_at_end"] == 0
    assert o["losses_finite"] and o["moved"] > 0
