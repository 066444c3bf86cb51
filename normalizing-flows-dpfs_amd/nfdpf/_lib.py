"""ctypes binding of libnfdpf.so (C ABI: include/nfdpf.h).

The library is built in-tree (``normalizing-flows-dpfs_amd/libnfdpf.so``) by
``__graft_entry__.build()`` / ``make -C normalizing-flows-dpfs_amd/csrc``.  There is no
fallback: if the library is missing, or no HIP device is present, every op raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_int32, c_int64, c_uint64, c_void_p

import torch  # noqa: F401  (load torch's HIP runtime first; libnfdpf binds to the same one)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("NFDPF_LIB", os.path.join(PKG_DIR, "libnfdpf.so"))

NFDPF_OK, NFDPF_EINVAL, NFDPF_ELAUNCH = 0, 1, 2
MEAS = {"cos": 0, "CRNVP": 1, "NN": 2, "gaussian": 3, "external": 4}
MEAS_EXTERNAL = 4
RESAMPLE = {"soft": 0, "ot": 1}
RNG_DEVICE, RNG_HOST = 0, 1
DYN_NONE, DYN_REALNVP, DYN_MAF = 0, 1, 2


class FilterDesc(Structure):
    """Mirror of ``nfdpf_filter_desc`` (include/nfdpf.h); field order must match."""

    _fields_ = [
        ("B", c_int32), ("N", c_int32), ("T", c_int32), ("E", c_int32),
        ("B_global", c_int32), ("t", c_int32), ("phase", c_int32),
        ("row_base", c_int64),
        ("nf_dyn", c_int32), ("nf_cond", c_int32), ("measurement", c_int32), ("resampler", c_int32),
        ("rng_mode", c_int32), ("force_resample", c_int32), ("n_flows", c_int32), ("hidden", c_int32),
        ("defer_norm", c_int32), ("split_nets", c_int32),
        ("alpha", c_float), ("pos_noise", c_float), ("dens_const", c_float), ("meas_prior_std", c_float),
        ("seed", c_uint64),
        ("dyn_params", c_void_p), ("cond_params", c_void_p), ("pe_params", c_void_p), ("meas_params", c_void_p),
        ("enc", c_void_p), ("vel", c_void_p), ("lin", c_void_p), ("host_noise", c_void_p),
        ("host_offsets", c_void_p), ("x_prev", c_void_p), ("p_prev", c_void_p),
        ("x_prev_rs", c_int64), ("p_prev_rs", c_int64),
        ("ess_all", c_void_p), ("gate", c_void_p), ("ot_x", c_void_p), ("lik_ext", c_void_p),
        ("hist_x", c_void_p), ("hist_p", c_void_p), ("hist_noise", c_void_p), ("hist_lik", c_void_p),
        ("hist_jac", c_void_p), ("hist_prior", c_void_p), ("hist_idx", c_void_p),
        ("ess_out", c_void_p), ("lw_sum", c_void_p), ("pred", c_void_p), ("scratch", c_void_p),
        ("prof_events", c_void_p),
        ("ess_local", c_int32),
        ("prof_front", c_int32),
        ("pass_gate", c_int32),
        ("pass_gates", c_void_p), ("pass_flags", c_void_p), ("pass_obs", c_void_p),
        ("meas_mfma", c_int32),
        ("pass_plan", c_void_p),
        ("gate_peers", c_void_p), ("gate_world", c_int32), ("gate_rank", c_int32),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "nfdpf_version": (c_int, []),
    "nfdpf_last_error": (c_char_p, []),
    "nfdpf_cond_stack": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int64,
                                 c_int, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_cond_stack_backward_workspace": (c_int64, [c_int, c_int, c_int, c_int, c_int64]),
    "nfdpf_cond_stack_backward": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int,
                                          c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p]),
    "nfdpf_ot_transport_backward": (c_int, [c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p,
                                            c_void_p]),
    "nfdpf_soft_resample_backward_workspace": (c_int64, [c_int, c_int]),
    "nfdpf_soft_resample_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                             c_float, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_cos_measurement_backward_workspace": (c_int64, [c_int, c_int]),
    "nfdpf_cos_measurement_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_nn_measurement_backward_workspace": (c_int64, [c_int, c_int]),
    "nfdpf_nn_measurement_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_particle_encoder": (c_int, [c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p]),
    "nfdpf_maf_stack": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                                c_void_p]),
    "nfdpf_soft_resample": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int64,
                                    c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_ot_workspace_bytes": (c_int64, [c_int, c_int]),
    "nfdpf_ot_stats": (c_int, [c_void_p, c_void_p]),
    "nfdpf_ot_resample": (c_int, [c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_int, c_int64,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int, c_void_p]),
    "nfdpf_ot_resample_rs": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int, c_float, c_float, c_float,
                                     c_int, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_int, c_void_p]),
    "nfdpf_ot_history_bytes": (c_int64, [c_int, c_int, c_int]),
    "nfdpf_ot_sinkhorn_local": (c_int, [c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_int, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "nfdpf_ot_sinkhorn_finish": (c_int, [c_void_p, c_int, c_int, c_float, c_float, c_float, c_int, c_int64, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p]),
    "nfdpf_ess_gate":(c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_maf_stack_backward_workspace": (c_int64, [c_int, c_int, c_int, c_int64]),
    "nfdpf_maf_stack_backward": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_pseudo_lik_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                         c_void_p, c_void_p]),
    "nfdpf_pseudo_lik_workspace": (c_int64, [c_int, c_int, c_int, c_int]),
    "nfdpf_pseudo_lik_check": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_pseudo_lik_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_rqs": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_float, c_float,
                          c_float, c_float, c_int, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    "nfdpf_split_fault": (c_int, [c_int, c_void_p]),
    "nfdpf_normalize_log_probs": (c_int, [c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p]),
    "nfdpf_cglow_params_size": (c_int64, [c_int]),
    "nfdpf_cglow_measurement": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int,
                                        c_int, c_void_p, c_int64, c_void_p]),
    "nfdpf_cglow_flow": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "nfdpf_cglow_backward_workspace": (c_int64, [c_int64]),
    "nfdpf_cglow_measurement_backward": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_int64,
                                                 c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_void_p, c_void_p]),
    "nfdpf_cglow_flow_backward": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_measurement": (c_int, [c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                                  c_float, c_void_p, c_void_p]),
    "nfdpf_particle_init": (c_int, [c_void_p, c_int, c_int, c_float, c_int, c_uint64, c_int64, c_void_p, c_void_p,
                                    c_void_p]),
    "nfdpf_cascade_row_sum": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_filter_step": (c_int, [POINTER(FilterDesc), c_void_p]),
    "nfdpf_filter_tiled_workspace_bytes": (c_int64, [c_int, c_int, c_int]),
    "nfdpf_filter_tiled_tiles": (c_int, [c_int]),
    "nfdpf_filter_tiled_fused": (c_int, [POINTER(FilterDesc)]),
    "nfdpf_filter_desc_size": (c_int64, []),
    "nfdpf_filter_tiled_init": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_host_mapped_alloc": (c_int, [c_int64, c_void_p, c_void_p]),
    "nfdpf_host_mapped_free": (c_int, [c_void_p]),
    "nfdpf_ess_row_terms": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_ess_gate_terms": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_gate_xchg_bytes": (c_int64, [c_int]),
    "nfdpf_gate_xchg_alloc": (c_int, [c_int64, c_void_p, c_void_p]),
    "nfdpf_gate_xchg_open": (c_int, [c_void_p, c_void_p]),
    "nfdpf_gate_xchg_close": (c_int, [c_void_p]),
    "nfdpf_gate_xchg_free": (c_int, [c_void_p]),
    "nfdpf_filter_init": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_uint64,
                                  c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nfdpf_filter_pass_supported": (c_int, [POINTER(FilterDesc)]),
    "nfdpf_filter_pass_workspace_bytes": (c_int64, [c_int, c_int, c_int]),
    "nfdpf_filter_pass_tiled": (c_int, [POINTER(FilterDesc), c_void_p, c_void_p]),
    "nfdpf_filter_step_tiled": (c_int, [POINTER(FilterDesc), c_void_p, c_void_p]),
    "nfdpf_ess_gate_tiled": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_ess_gate_tiled_batch": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "nfdpf_pass_verify": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
}

_lib = None


class NfdpfError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libnfdpf.so and declare every C-ABI signature (no device needed)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NfdpfError(f"libnfdpf.so not found at {path}: build it with "
                         f"`python -c 'import __graft_entry__ as g; g.build()'` or `make -C {PKG_DIR}/csrc`")
    lib = ctypes.CDLL(path)
    # NFDPF_LIB_PARTIAL=1 (experiment builds of older sources, scripts/archive/exp_run.sh only): skip
    # entry points the library lacks; otherwise a missing symbol is an error
    partial = os.environ.get("NFDPF_LIB_PARTIAL") == "1"
    for name, (res, args) in SIGNATURES.items():
        if partial and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if hasattr(lib, "nfdpf_filter_desc_size"):  # the struct mirror must match the library's
        n = int(lib.nfdpf_filter_desc_size())
        if n != ctypes.sizeof(FilterDesc):
            raise NfdpfError(f"{path}: nfdpf_filter_desc is {n} bytes, nfdpf._lib.FilterDesc "
                             f"{ctypes.sizeof(FilterDesc)} (stale library or binding)")
    elif not partial:
        raise NfdpfError(f"{path}: no nfdpf_filter_desc_size (stale library)")
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def check(rc: int, what: str):
    if rc != NFDPF_OK:
        msg = lib().nfdpf_last_error().decode(errors="replace")
        raise NfdpfError(f"{what} failed (rc={rc}): {msg}")


def check_split_fault(what: str = "tiled filter step", device=None):
    """Raise if a wave-pair hand-off of the tiled step gave up on its partner (csrc/split.hpp
    kSpinCap) since the last check: that launch ran on stale data.  Read in order on the
    current stream of ``device`` (where the launches ran), then synchronises that stream."""
    n = lib().nfdpf_split_fault(1, stream_ptr(device))
    if n != 0:
        raise NfdpfError(f"{what}: {n} wave-pair hand-off(s) timed out on the device (outputs invalid)"
                         if n > 0 else f"{what}: could not read the device fault counter")


def require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise NfdpfError(f"{what}: the nfdpf hot path runs on the HIP device only (got a {t.device} tensor)")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()
