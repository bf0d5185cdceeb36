"""ctypes binding of libppo_hip.so (the C ABI declared in include/ppo_hip.h).

There is no CPU fallback: if the library is missing or fails to load, every op
raises.  Device memory comes from torch's caching allocator; the library only
sees raw pointers, sizes and the current HIP stream.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PPO_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libppo_hip.so"))

c_int, c_ll, c_ull, c_f, c_d, c_p = (ctypes.c_int, ctypes.c_longlong, ctypes.c_ulonglong, ctypes.c_float,
                                     ctypes.c_double, ctypes.c_void_p)

# name -> argtypes (all return int status unless listed in _RESTYPES)
SIGNATURES = {
    "ppo_abi_version": [],
    "ppo_last_error": [],
    "ppo_prof_enable": [ctypes.c_char_p, c_int],
    "ppo_prof_collect": [c_p],
    "ppo_prof_collect_one": [c_int, c_p],
    # gae.hip
    "ppo_gae_partials_count": [c_int],
    "ppo_compute_returns": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_d, c_d, c_int, c_int, c_p],
    "ppo_gae_scan_partials_count": [c_int],
    "ppo_compute_returns_scan": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_d, c_d, c_int, c_int, c_p],
    "ppo_adv_diff_partials_count": [c_ll],
    "ppo_adv_diff": [c_p, c_p, c_p, c_p, c_ll, c_p],
    "ppo_adv_finalize": [c_p, c_int, c_d, c_p, c_p],
    "ppo_adv_normalize": [c_p, c_ll, c_p, c_p],
    # storage.hip
    "ppo_copy": [c_p, c_p, c_ll, c_p],
    "ppo_fill_f32": [c_p, c_ll, c_f, c_p],
    "ppo_storage_insert_scalars": [c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "ppo_gather_rows": [c_p, c_p, c_p, c_ll, c_ll, c_p],
    "ppo_gather_env_columns": [c_p, c_p, c_p, c_int, c_int, c_int, c_ll, c_p],
    "ppo_gather_f16_to_f32": [c_p, c_p, c_p, c_ll, c_ll, c_p],
    "ppo_synth_env_step": [c_p, c_int, c_ll, c_p, c_p, c_p, c_ull, c_ull, c_f, c_p],
    "ppo_cartpole_step": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_ull, c_ull, c_int, c_p],
    # gemm.hip
    "ppo_packed_weights_size": [c_int],
    "ppo_packed_offsets": [c_int, c_p],
    "ppo_pack_weights": [c_p, c_p, c_p, c_int, c_p, c_p],
    "ppo_conv1_fwd": [c_p, c_int, c_p, c_ll, c_int, c_int, c_p, c_p, c_p, c_p],
    "ppo_conv1_fwd_mask": [c_p, c_int, c_p, c_ll, c_int, c_int, c_p, c_p, c_p, c_p, c_p],
    "ppo_conv1_fwd_f32": [c_p, c_p, c_ll, c_int, c_p, c_p, c_p, c_p, c_p],
    "ppo_conv1_fwd_rgb": [c_p, c_p, c_ll, c_int, c_p, c_d, c_p, c_p, c_p, c_p, c_p],
    "ppo_conv1_wgrad_f32": [c_p, c_p, c_p, c_ll, c_int, c_int, c_p, c_p, c_p],
    "ppo_conv1_wgrad_rgb": [c_p, c_p, c_p, c_ll, c_int, c_p, c_d, c_int, c_p, c_p, c_p],
    "ppo_conv2_fwd": [c_p, c_int, c_p, c_p, c_p, c_p],
    "ppo_conv2_fwd_mask": [c_p, c_int, c_p, c_p, c_p, c_p, c_p],
    "ppo_conv3_fwd": [c_p, c_int, c_p, c_p, c_p, c_p],
    "ppo_trunk_fwd": [c_p, c_p, c_ll, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "ppo_linear_relu_fwd": [c_p, c_int, c_int, c_p, c_p, c_int, c_p, c_p],
    "ppo_fc_fwd": [c_p, c_int, c_p, c_p, c_int, c_p, c_int, c_p],
    "ppo_fc_fwd_ws_bytes": [c_int, c_int],
    "ppo_fc_fwd_ws": [c_p, c_int, c_p, c_p, c_int, c_p, c_int, c_p, c_ll, c_p],
    "ppo_linear_dgrad_mask": [c_p, c_int, c_int, c_p, c_int, c_p, c_p, c_p],
    "ppo_conv3_fwd_mask": [c_p, c_int, c_p, c_p, c_p, c_p, c_p],
    "ppo_fc_dgrad_bits": [c_p, c_int, c_int, c_p, c_p, c_p, c_p],
    "ppo_conv3_dgrad": [c_p, c_int, c_p, c_p, c_p, c_p],
    "ppo_conv3_dgrad_bits_ok": [],
    "ppo_conv3_dgrad_bits": [c_p, c_int, c_p, c_p, c_p, c_p],
    "ppo_conv2_dgrad": [c_p, c_int, c_p, c_p, c_p, c_p],
    "ppo_conv2_dgrad_bits_ok": [],
    "ppo_conv2_dgrad_bits": [c_p, c_int, c_p, c_p, c_p, c_p],
    "ppo_wgrad_splits": [c_ll, c_int, c_int, c_int],
    "ppo_conv1_wgrad": [c_p, c_p, c_int, c_p, c_ll, c_int, c_int, c_int, c_p, c_p, c_p],
    "ppo_conv2_wgrad": [c_p, c_p, c_int, c_int, c_p, c_p, c_p],
    # probe.hip (CU-contention diagnostics)
    "ppo_probe_side_kernel": [c_int, c_int, c_ll, c_p, c_p],
    "ppo_probe_now": [c_p, c_p],
    "ppo_conv3_wgrad": [c_p, c_p, c_int, c_int, c_p, c_p, c_p],
    "ppo_linear_wgrad": [c_p, c_p, c_int, c_int, c_int, c_int, c_p, c_p, c_p],
    "ppo_wgrad_reduce": [c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p, c_p, c_f, c_int, c_p],
    "ppo_colsum": [c_p, c_ll, c_int, c_ll, c_p, c_f, c_int, c_p],
    "ppo_tune_set": [ctypes.c_char_p, c_int],
    "ppo_tune_get": [ctypes.c_char_p],
    # heads.hip
    "ppo_heads_act": [c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p, c_int, c_p, c_ull, c_ull, c_int, c_p, c_p, c_p,
                      c_p, c_p, c_p],
    "ppo_heads_train_blocks": [c_int],
    "ppo_heads_train": [c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p, c_int, c_p, c_ll, c_p, c_p, c_p, c_p, c_p, c_f,
                        c_f, c_f, c_f, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p],
    "ppo_linear_fwd_ex": [c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_int, c_p, c_int, c_int, c_p],
    "ppo_linear_dgrad_ex": [c_p, c_int, c_int, c_p, c_int, c_p, c_int, c_int, c_p, c_p],
    "ppo_transpose": [c_p, c_int, c_int, c_p, c_p],
    "ppo_gru_step_fwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "ppo_gru_cell_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p],
    "ppo_gru_step_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_p],
    "ppo_gru_variant_set": [c_int],
    "ppo_gru_variant_get": [],
    "ppo_gru_persist_set": [c_int],
    "ppo_gru_persist_get": [],
    "ppo_gru_persist_timeouts": [c_p],
    "ppo_gru_persist_spin_set": [c_int],
    "ppo_gru_seq_counters": [c_int],
    "ppo_gru_seq_fwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "ppo_gru_seq_fwd_ws": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                           c_p],
    "ppo_gru_seq_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p],
    "ppo_gru_seq_bwd_ws": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p,
                           c_p, c_p],
    "ppo_gru_step_bwd_cell": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p],
    "ppo_gru_pack": [c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p],
    "ppo_concat_cols": [c_p, c_p, c_ll, c_int, c_p, c_int, c_int, c_int, c_p],
    "ppo_rec_indices": [c_p, c_int, c_int, c_int, c_p, c_p],
    "ppo_heads_reduce": [c_p, c_p, c_p, c_int, c_int, c_int, c_p, c_p, c_p, c_p, c_p, c_d, c_f, c_int, c_p],
    "ppo_mean_f32": [c_p, c_ll, c_p, c_p],
    # obs.hip
    "ppo_obs_preprocess": [c_p, c_ll, c_int, c_int, c_int, c_p, c_d, c_int, c_p, c_ll, c_p],
    "ppo_frame_stack": [c_p, c_int, c_int, c_ll, c_p, c_p, c_int, c_p],
    # optim.hip
    "ppo_grad_partials_count": [c_ll],
    "ppo_grad_sumsq": [c_p, c_ll, c_f, c_p, c_p],
    "ppo_clip_adam": [c_p, c_p, c_p, c_p, c_ll, c_p, c_f, c_d, c_d, c_d, c_d, c_d, c_ll, c_p, c_p],
    "ppo_clip_adam_guarded": [c_p, c_p, c_p, c_p, c_ll, c_p, c_f, c_d, c_d, c_d, c_d, c_d, c_ll, c_p, c_p, c_p, c_p,
                              c_p],
}
_RESTYPES = {"ppo_last_error": ctypes.c_char_p, "ppo_packed_weights_size": c_ll, "ppo_fc_fwd_ws_bytes": c_ll}
# functions whose int return value is a result, not a status
_VALUE_FUNCS = {"ppo_abi_version", "ppo_gae_partials_count", "ppo_gae_scan_partials_count", "ppo_adv_diff_partials_count",
                "ppo_packed_weights_size", "ppo_fc_fwd_ws_bytes", "ppo_wgrad_splits", "ppo_heads_train_blocks", "ppo_grad_partials_count",
                "ppo_conv2_dgrad_bits_ok", "ppo_conv3_dgrad_bits_ok", "ppo_tune_get",
                "ppo_gru_persist_get", "ppo_gru_persist_timeouts", "ppo_gru_seq_counters"}

_LIB = None


def lib():
    """Load libppo_hip.so (raises if it is missing: there is no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libppo_hip.so not found at {LIB_PATH}: build it with `make -C ppo-dash_amd` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            if name.startswith("ppo_probe_") and not hasattr(L, name):
                continue   # diagnostics only: an older library (same-box A/B builds) may lack a probe
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, c_int)
        _LIB = L
    return _LIB


class HipError(RuntimeError):
    pass


def call(name, *args):
    fn = getattr(lib(), name)
    rc = fn(*args)
    if name in _VALUE_FUNCS or name in _RESTYPES:
        return rc
    if rc != 0:
        msg = lib().ppo_last_error().decode(errors="replace")
        raise HipError(f"{name} failed ({rc}): {msg}")
    return rc


def stream():
    return torch.cuda.current_stream().cuda_stream


def ptr(t, dtype=None, name="tensor"):
    """Raw device pointer of a contiguous CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be on the MI355X (got {t.device}); the HIP engine has no CPU path")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    return t.data_ptr()


def require_device():
    if not torch.cuda.is_available():
        raise RuntimeError("no MI355X visible: the a2c_ppo_acktr HIP engine needs a GPU (there is no CPU fallback)")
