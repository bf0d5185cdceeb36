"""CPU-only checks: the C-ABI library loads and exports every symbol the header
declares, the ctypes table matches the header, host-side invariants."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ppo_hip.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*[a-z_][a-z_0-9 \t\*]*?\b(ppo_[a-z0-9_]+)\s*\(", src, re.M)))


def test_header_has_entry_points():
    syms = header_symbols()
    assert len(syms) >= 35
    assert "ppo_compute_returns" in syms and "ppo_clip_adam" in syms


def test_library_exports_every_declared_symbol():
    from a2c_ppo_acktr import _hip
    lib = _hip.lib()   # loads without a GPU; no compute calls are made
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.ppo_abi_version() == 3


def test_library_resolves_every_symbol_at_load():
    """RTLD_NOW: a symbol the library references but nothing defines (e.g. a helper
    left with internal linkage in one source and declared extern in another) fails
    here instead of at the first call on a GPU box"""
    import ctypes
    import os
    from a2c_ppo_acktr import _hip
    ctypes.CDLL(_hip.LIB_PATH, mode=os.RTLD_NOW)


def test_ctypes_table_matches_header():
    from a2c_ppo_acktr import _hip
    assert sorted(_hip.SIGNATURES) == header_symbols()
    src = open(HEADER).read()
    for name, args in _hip.SIGNATURES.items():
        decl = re.search(name + r"\s*\(([^)]*)\)", src).group(1).strip()
        n = 0 if decl in ("", "void") else decl.count(",") + 1
        assert n == len(args), (name, n, len(args))


def test_host_only_queries():
    from a2c_ppo_acktr import _hip
    assert _hip.call("ppo_gae_partials_count", 4096) == 16
    # f32 segments, each followed by its three bf16 planes (1.5x its size in floats)
    assert _hip.call("ppo_packed_weights_size", 512) == (64 * 512 + 32 * 576 + 2 * 512 * 1568 + 64 * 288
                                                         + 4 * 32 * 256) * 5 // 2
    z = _hip.call("ppo_wgrad_splits", 65536 * 400, 1, 2048, 16)
    assert 1 <= z <= 4096
    assert _hip.call("ppo_heads_train_blocks", 65536) == 65536 // 128


def test_tune_knobs_accept_listed_values_only():
    """ppo_tune_set (include/ppo_hip.h, run-time knobs): each key takes its listed
    values, anything else is refused with PPO_EARG and leaves the knob unchanged;
    unknown keys read -1.  Host-only: no GPU call."""
    from a2c_ppo_acktr import _hip
    listed = {"conv1_fwd": (0, 9), "conv1_wgrad": (9, 10, 8, 5), "x9": (1, 0, 2), "fc_splitk": (4, 0, 8),
              "fc_splitk_tile": (1, 0), "rgb_aff": (1, 0), "stagger": (2, 0, 15), "products": (6, 9, 1)}
    refused = {"conv1_fwd": (1, 2, 10), "conv1_wgrad": (0, 7, 11), "x9": (-1, 3), "fc_splitk": (-1, 9),
               "fc_splitk_tile": (2,), "rgb_aff": (2,), "stagger": (16, 255, -1), "products": (0, 2, 5)}
    for key, vals in listed.items():
        k = key.encode()
        old = _hip.call("ppo_tune_get", k)
        assert old == vals[0], (key, old)   # the documented default
        try:
            for v in vals:
                _hip.call("ppo_tune_set", k, v)
                assert _hip.call("ppo_tune_get", k) == v
            _hip.call("ppo_tune_set", k, old)
            for v in refused[key]:
                with pytest.raises(_hip.HipError, match="1001"):
                    _hip.call("ppo_tune_set", k, v)
                assert _hip.call("ppo_tune_get", k) == old
        finally:
            _hip.call("ppo_tune_set", k, old)
    assert _hip.call("ppo_tune_get", b"no_such_knob") == -1
    with pytest.raises(_hip.HipError):
        _hip.call("ppo_tune_set", b"no_such_knob", 0)


def test_u8_decode_exact_for_all_codes():
    from oracle import ppo_oracle as O
    lib = O._lib()
    lib.oracle_decode_u8_fma.restype = ctypes.c_float
    lib.oracle_decode_u8_fma.argtypes = [ctypes.c_uint]
    got = np.array([lib.oracle_decode_u8_fma(u) for u in range(256)], np.float32)
    ref = np.arange(256, dtype=np.uint8).astype(np.float32) / np.float32(255.0)
    assert np.array_equal(got, ref)


def test_api_surface_imports():
    """run.py's imports (T/run.py:15-23) resolve against the drop-in package."""
    from a2c_ppo_acktr import algo, utils  # noqa: F401
    from a2c_ppo_acktr.algo import gail  # noqa: F401
    from a2c_ppo_acktr.arguments import get_args  # noqa: F401
    from a2c_ppo_acktr.model import CNNBase, Policy  # noqa: F401
    from a2c_ppo_acktr.storage import RolloutStorage  # noqa: F401
    from a2c_ppo_acktr.utils import get_render_func, get_vec_normalize  # noqa: F401
    assert hasattr(algo, "PPO") and hasattr(algo, "A2C_ACKTR")


def test_policy_construction_matches_reference_init():
    """Same seed + construction order -> the reference's initial parameters."""
    import torch
    from conftest import golden
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("cnn_update.npz")
    nt = torch.get_num_threads()
    torch.set_num_threads(1)   # as T/run.py:55; orthogonal_'s QR depends on the thread count
    torch.manual_seed(1)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": 64})
    assert [n for n, _ in pol.named_parameters()] == [str(x) for x in d["names"]]
    init = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy()
    assert np.array_equal(init, d["init_params"])
    g = golden("gru_eval.npz")
    torch.manual_seed(11)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": 32},
                   vector_obs_len=14)
    assert [n for n, _ in pol.named_parameters()] == [str(x) for x in g["names"]]
    assert np.array_equal(torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy(), g["params"])
    # gru_update.npz: the recurrent policy of the recorded update, and the default
    # generator's state after construction (the replay's sampling / randperm draws
    # start from it: tests/test_gpu_parity.py test_recurrent_iteration_replays_reference)
    u = golden("gru_update.npz")
    torch.manual_seed(31)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": 32},
                   vector_obs_len=14)
    assert np.array_equal(torch.get_rng_state().numpy(), u["rng_after_init"])
    gw = torch.Generator().manual_seed(32)
    with torch.no_grad():
        pol.dist.linear.weight.mul_(40.0)
        pol.base.gru.bias_ih_l0.copy_(torch.rand(96, generator=gw) * 0.6 - 0.3)
        pol.base.gru.bias_hh_l0.copy_(torch.rand(96, generator=gw) * 0.6 - 0.3)
    assert np.array_equal(torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy(), u["init_params"])
    # the production-size replays: c3's H = 512 CNN and c5's
    # H = 256 GRU + 14 vector obs, constructed in the reference's order
    for name in ("cnn_update_h512.npz", "cnn_update_wide.npz"):
        c = golden(name)
        torch.manual_seed(1)
        pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": 512})
        assert np.array_equal(torch.get_rng_state().numpy(), c["rng_after_init"]), name
        assert np.array_equal(torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy(), c["init_params"])
    u = golden("gru_update_h256.npz")
    torch.manual_seed(31)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": 256},
                   vector_obs_len=14)
    assert np.array_equal(torch.get_rng_state().numpy(), u["rng_after_init"])
    gw = torch.Generator().manual_seed(32)
    with torch.no_grad():
        pol.dist.linear.weight.mul_(40.0)
        pol.base.gru.bias_ih_l0.copy_(torch.rand(768, generator=gw) * 0.6 - 0.3)
        pol.base.gru.bias_hh_l0.copy_(torch.rand(768, generator=gw) * 0.6 - 0.3)
    assert np.array_equal(torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy(), u["init_params"])
    torch.set_num_threads(nt)


def test_wide_fixture_observations_regenerate():
    """cnn_update_wide.npz stores its 129 x 128 observation frames as a generator
    seed: torch.randint on a seeded CPU generator reproduces them (byte sum and
    CRC-32 recorded at generation), as the GPU replay regenerates them."""
    import zlib
    import torch
    from conftest import golden
    d = golden("cnn_update_wide.npz")
    hidden, N, T, E, Mb = (int(x) for x in d["meta"])
    o = torch.randint(0, 256, (T + 1, N, 4, 84, 84), dtype=torch.uint8,
                      generator=torch.Generator().manual_seed(int(d["obs_seed"][0]))).numpy()
    assert [int(o.sum(dtype=np.int64)), zlib.crc32(o.tobytes())] == [int(x) for x in d["obs_check"]]


def test_update_linear_schedule_drives_optimizer_lr():
    import torch
    from a2c_ppo_acktr import utils
    from a2c_ppo_acktr.algo.ppo import FlatAdam
    opt = FlatAdam([torch.nn.Parameter(torch.zeros(3))], lr=1e-4, eps=1e-5)
    utils.update_linear_schedule(opt, 3, 10, 1e-4)
    assert abs(opt.param_groups[0]["lr"] - 7e-5) < 1e-12


def test_storage_host_errors():
    import torch
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    st = RolloutStorage(4, 2, (1,), [0], Discrete(2), 1)
    with pytest.raises(RuntimeError, match="move it to the MI355X"):
        st.compute_returns(torch.zeros(2, 1), True, 0.99, 0.95)
    assert st.half() is st and st.obs.dtype == torch.float32   # vector obs planes stay fp32
    img = RolloutStorage(2, 2, (4, 84, 84), [0], Discrete(2), 1)
    img.half()
    assert img.obs.dtype == torch.float16 and img.rewards.dtype == torch.float32 and img.actions.dtype == torch.int64
    u8 = RolloutStorage(2, 2, (4, 84, 84), [0], Discrete(2), 1, obs_dtype=torch.uint8)
    assert u8.half().obs.dtype == torch.uint8
    with pytest.raises(AssertionError):
        next(st.feed_forward_generator(torch.zeros(4, 2, 1), 100))


def test_bf16x3_split_is_exact():
    """The exact three-way bf16 split behind the matrix-core fp32 paths
    (csrc/common.h split_bf16x3): v == hi + mid + lo bit for bit,
    each part a round-to-nearest-even bf16 of the remaining residual (for
    |v| > ~1e-30; below that lo is subnormal and the split is off by < 2^-133)."""
    import numpy as np

    def rne(v):
        u = v.view(np.uint32).astype(np.uint64)
        return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32)

    def tof(h):
        return (h.astype(np.uint32) << 16).view(np.float32)

    rng = np.random.default_rng(0)
    for scale in (1e-30, 1e-6, 1e-3, 0.05, 1.0, 1e3, 1e30):
        v = (rng.standard_normal(500_000) * scale).astype(np.float32)
        hi = rne(v)
        r1 = (v - tof(hi)).astype(np.float32)
        mid = rne(r1)
        r2 = (r1 - tof(mid)).astype(np.float32)
        lo = rne(r2)
        back = tof(hi).astype(np.float64) + tof(mid) + tof(lo)
        if scale >= 1e-20:
            assert np.array_equal(back, v.astype(np.float64)), scale
        else:   # lo falls into the subnormal range: off by at most its spacing, 2^-133
            assert np.abs(back - v).max() <= 2.0 ** -133, scale


def test_gemm_plane_swizzle_conflict_free():
    """igemm_x9.h pl_off: the ds_read_b128 fragment groups, the split-at-staging
    non-KC writes and the KC writes are all free of LDS bank conflicts (exhaustive
    over a 256-row tile, tools/swizzle_check.py restates the function)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "ppo-dash_amd", "csrc", "igemm_x9.h")).read()
    assert "(row ^ ((row >> 4) & 1)) * 32 + 8 * (q ^ ((H4 >> (4 * ((row >> 2) & 3))) & 3))" in src
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "swizzle_check.py")], capture_output=True,
                         text=True, check=True).stdout
    assert "reads 1 non-KC writes 1 KC writes 1" in out


def test_conv_row_tiles_cover_every_output_once():
    """Row-tile maps of the standalone conv forwards (gemm.hip conv2_fwd_x9c_body
    with MT = 5 + conv2_fwd_lone_kernel; conv3_fwd_c3_kernel + conv3_fwd_lone_kernel),
    restated: every output pixel is computed exactly once, dummy rows write nothing,
    and a 16-row tile's phase-grid rows collide in residue mod 16 (a bank conflict of
    the fragment read) at most 2-way.  conv2: v = 10 oy + ox over the 9 x 10 phase
    grid, m = 9 oy + ox; the lone pixel is v = 80 (m = 72).  conv3: compact rows
    m = 7 oy + ox < 48 on three tiles, m = 48 lone."""
    vtab = [[None] * 16 for _ in range(5)]
    for tid in range(16):
        t = 0
        for v in range(tid, 89, 16):
            if v % 10 != 9 and t < 5:
                vtab[t][tid] = v
                t += 1
        if t == 4:   # residues 9, 11, 13, 15 take v = 82 .. 88
            vtab[4][tid] = 82 + (tid - 9)
            t = 5
        assert t == 5
    outs = [9 * (v // 10) + v % 10 for row in vtab for v in row] + [72]
    assert sorted(outs) == list(range(81))
    for row in vtab:
        res = [v % 16 for v in row]
        assert max(res.count(r) for r in set(res)) <= 2
    conv3 = [16 * t + i for t in range(3) for i in range(16)] + [48]
    assert sorted(conv3) == list(range(49))
    # tap pixels of the compact rows stay on the 9 x 9 grid (no pad row reached)
    for m in range(48):
        oy, ox = divmod(m, 7)
        assert 9 * oy + ox + 9 * 2 + 2 <= 80


def test_bench_pmc_lookups_tolerate_other_workloads():
    """bench.py's PMC lookups (MFMA utilisation, shader clock, HBM traffic) return
    empty results — never raise — for a workload the committed profiles do not hold."""
    import bench
    util, clk, src = bench.pmc_mfma("no such workload")
    assert util == {} and clk == {}
    traffic, tsrc = bench.pmc_traffic("conv2_fwd", "no such workload")
    assert traffic is None
