"""ctypes binding of libsfx.so (the C ABI declared in include/sfx.h).

The library is the product path: there is no CPU fallback.  If libsfx.so is absent,
importing this module raises; if no HIP device is present, compute calls fail loudly
from the HIP runtime.  ``torch`` is imported first so the process uses the HIP
runtime torch already loaded (libamdhip64.so.7), not a second copy.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (load torch's HIP runtime before libsfx.so)

LIB_PATH = os.environ.get("SFX_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsfx.so"))

# name -> (restype, argtypes); every function declared in include/sfx.h
_VP, _I, _D, _F = C.c_void_p, C.c_int, C.c_double, C.c_float
_IP, _FP = C.POINTER(C.c_int), C.POINTER(C.c_float)
SIGNATURES = {
    "sfx_version": (C.c_char_p, []),
    "sfx_last_error": (C.c_char_p, []),
    "sfx_create": (_I, [C.POINTER(_VP), _I, _I, _I, _I, _IP, _I, _I, _I, _I, _VP]),
    "sfx_destroy": (_I, [_VP]),
    "sfx_set_stream": (_I, [_VP, _VP]),
    "sfx_set_graphs": (_I, [_VP, _I]),
    "sfx_head_numel": (_I, [_VP]),
    "sfx_set_adam": (_I, [_VP, _D, _D, _D, _D, _D, _D, _D]),
    "sfx_load_head": (_I, [_VP, _I, _I, _FP]),
    "sfx_get_head": (_I, [_VP, _I, _I, _FP]),
    "sfx_load_adam": (_I, [_VP, _I, _FP, _FP, _I]),
    "sfx_get_adam": (_I, [_VP, _I, _FP, _FP, _IP]),
    "sfx_load_w": (_I, [_VP, _I, _FP]),
    "sfx_get_w": (_I, [_VP, _I, _FP, _FP, _FP]),
    "sfx_load_w_state": (_I, [_VP, _I, _FP, _FP, _FP]),
    "sfx_w_ptr": (_I, [_VP, _I, C.POINTER(_VP)]),
    "sfx_gpi": (_I, [_VP, _VP, _I, _VP, _VP, _VP, _VP, _VP]),
    "sfx_successors": (_I, [_VP, _VP, _I, _I, _VP]),
    "sfx_select_action": (_I, [_VP, _VP, _I, _I, _VP, _VP]),
    "sfx_test_actions": (_I, [_VP, _VP, _I, _VP, _I, _VP, _VP]),
    "sfx_nonfinite": (_I, [_VP, _VP, _I]),
    "sfx_runner_nonfinite": (_I, [_VP, _VP]),
    "sfx_test_reward_updates": (_I, [_VP, _I, _VP, _VP, _VP, _I, C.c_double, C.c_double, _VP]),
    "sfx_update": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP]),
    "sfx_update_all": (_I, [_VP, _VP, _VP, _VP, _VP, _VP, _I, _VP]),
    "sfx_update_all_select": (_I, [_VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, _VP, _I, _VP, _VP, _I, _VP, _F, _VP, _F]),
    "sfx_settle": (_I, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int64)]),
    "sfx_lms": (_I, [_VP, _I, _VP, _VP, _F]),
    "sfx_lms_value": (_I, [_VP, _I, _VP, _F, _F]),
    "sfx_host_alloc": (_I, [C.c_size_t, C.POINTER(_VP)]),
    "sfx_host_free": (_I, [_VP]),
    "sfx_step_all": (_I, [_VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _I, _VP, _VP, _F, _VP, _I, _I, _VP]),
    "sfx_step_finish": (_I, [_VP, C.POINTER(C.c_int64)]),
    "sfx_debug_force_rerun": (_I, [_VP, _I]),
    "sfx_set_spec_rounds": (_I, [_VP, _I]),
    "sfx_step_stats": (_I, [_VP] + [C.POINTER(C.c_longlong)] * 4),
    "sfx_graph_stats": (_I, [_VP] + [C.POINTER(C.c_longlong)] * 3),
    "sfx_skip_stats": (_I, [_VP, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong), _I]),
    "sfx_set_precision": (_I, [_VP, _I]),
    "sfx_get_precision": (_I, [_VP]),
    "sfx_set_huber": (_I, [_VP, _F]),
    "sfx_replay_put": (_I, [_VP] * 5 + [C.c_longlong] + [_VP] * 4 + [_I, _I]),
    "sfx_replay_put_gather": (_I, [_VP] * 6 + [C.c_longlong] + [_VP] * 8 + [_I] + [_VP] * 5 + [_I, _I]),
    "sfx_replay_gather": (_I, [_VP] * 8 + [_I] + [_VP] * 5 + [_I, _I]),
    "sfx_get_huber": (_F, [_VP]),
    "sfx_set_target_update_ev": (_I, [_VP, _I]),
    "sfx_get_since_target": (_I, [_VP, _I, _IP]),
    "sfx_set_since_target": (_I, [_VP, _I, _I]),
    "sfx_sync_target": (_I, [_VP, _I]),
    "sfx_prof_enable": (_I, [_VP, _I]),
    "sfx_prof_collect": (_I, [_VP, _I, _IP, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "sfx_prof_reset": (_I, [_VP]),
    "sfx_synchronize": (_I, [_VP]),
    "sfx_runner_create": (_I, [C.POINTER(_VP), _VP, _I, _I, _F, _F, _F, _I, _I, C.c_ulonglong, _VP, _VP, _VP]),
    "sfx_runner_destroy": (_I, [_VP]),
    "sfx_runner_layout": (_I, [_VP, C.POINTER(C.c_int64)]),
    "sfx_runner_config": (_I, [_VP, _I, _I, _F]),
    "sfx_runner_device_replay": (_I, [_VP, _I]),
    "sfx_runner_set_task": (_I, [_VP, _I]),
    "sfx_runner_prefill": (_I, [_VP, _I]),
    "sfx_runner_run": (_I, [_VP, _I]),
    "sfx_runner_action": (_I, [_VP, C.POINTER(C.c_int64)]),
    "sfx_runner_stats": (_I, [_VP] + [C.POINTER(C.c_longlong)] * 3 + [C.POINTER(C.c_double)]),
    "sfx_runner_gate_timeout": (_I, [_VP, _D]),
    "sfx_runner_wait_timeout": (_I, [_VP, _D]),
    "sfx_runner_retried": (_I, [_VP, C.POINTER(C.c_longlong)]),
    "sfx_runner_ahead_stats": (_I, [_VP, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]),
    "sfx_runner_recomputed": (_I, [_VP, C.POINTER(C.c_longlong)]),
    "sfx_runner_warm": (_I, [_VP]),
    "sfx_runner_gpi_counters": (_I, [_VP, C.POINTER(C.c_longlong)]),
    "sfx_runner_record": (_I, [_VP, _I]),
    "sfx_runner_recorded": (_I, [_VP]),
    "sfx_runner_get_record": (_I, [_VP, _I, _VP, C.POINTER(C.c_int64)]),
    "sfx_comm_id_bytes": (_I, []),
    "sfx_comm_unique_id": (_I, [_VP]),
    "sfx_comm_init": (_I, [_VP, _VP, _I, _I]),
    "sfx_set_comm": (_I, [_VP, _VP, _I, _I]),
    "sfx_set_comm_host": (_I, [_VP, _VP, _VP, _I, _I]),
    "sfx_check_failures": (_I, [C.POINTER(C.c_longlong), _VP, _I]),
    "sfx_comm_state": (_I, [_VP, _VP]),
    "sfx_comm_size": (_I, [_VP, _VP, _VP, _VP, _VP]),
    "sfx_tsf_freeze_flows": (_I, [_VP, _I]),
    "sfx_debug_stall": (_I, [_VP, _D]),
    "sfx_shard_setup": (_I, [_VP, _I, _I]),
    "sfx_shard_begin": (_I, [_VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _F, _VP]),
    "sfx_shard_td_maxima": (_I, [_VP, _I, _VP]),
    "sfx_shard_td_update": (_I, [_VP, _I, _VP]),
    "sfx_shard_ver_maxima": (_I, [_VP, _I, _VP]),
    "sfx_shard_verify": (_I, [_VP, _VP, _VP, _VP]),
    "sfx_shard_select": (_I, [_VP, _I, _I, _I, _VP]),
    "sfx_shard_finish": (_I, [_VP, _I]),
    "sfx_shard_tsf_maxima": (_I, [_VP, _I, _VP, _I, _I, _VP]),
    "sfx_shard_tsf_update": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, _VP]),
    "sfx_shard_tsf_shared": (_I, [_VP, _I, _VP, _I]),
    "sfx_shard_tsf_select": (_I, [_VP, _VP, _I, _I, _VP]),
    "sfx_tsf_setup": (_I, [_VP, _I, _I, _F, _D, _D, _D, _D]),
    "sfx_tsf_load_g": (_I, [_VP, _I, _FP]),
    "sfx_tsf_get_g": (_I, [_VP, _I, _FP, _FP, _FP]),
    "sfx_tsf_load_h": (_I, [_VP, _FP]),
    "sfx_tsf_get_h": (_I, [_VP, _FP]),
    "sfx_tsf_load_g_state": (_I, [_VP, _I, _VP, _VP, _VP]),
    "sfx_tsf_get_h_state": (_I, [_VP, _I, _VP, _VP]),
    "sfx_tsf_load_h_state": (_I, [_VP, _I, _VP, _VP]),
    "sfx_tsf_update": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP]),
    "sfx_tsf_test_action": (_I, [_VP, _VP, _VP, _VP, _VP]),
    "sfx_phi_setup": (_I, [_VP, _I, _I, _F]),
    "sfx_phi_numel": (_I, [_VP]),
    "sfx_phi_load": (_I, [_VP, _VP]),
    "sfx_phi_get": (_I, [_VP, _VP]),
    "sfx_phi_update": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP, _I, _I, _VP, _VP, _VP, _VP]),
    "sfx_tsf_test_update": (_I, [_VP, _VP, _VP, _VP, _VP, _F, _VP, _VP, _VP, _VP, _I] + [_F] * 7 + [_VP]),
    "sfx_tsf_test_actions": (_I, [_VP, _VP, _I, _VP, _I, _VP, _I, _VP]),
    "sfx_tsf_test_updates": (_I, [_VP, _I, _VP, _VP, _VP, _VP, _VP, _VP, _I, _VP, _I, _VP, _I, _VP, _F, _F, _F, _VP]),
}

# env callbacks of sfx_runner_create (include/sfx.h)
ENV_RESET_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_float))
ENV_STEP_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float),
                          C.POINTER(C.c_float), C.POINTER(C.c_int))


# host all-reduce(MAX) callback of sfx_set_comm_host: (ctx, float* host buffer, count) -> 0 on success
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int32), C.c_int)


class SFXError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsfx.so not found at {LIB_PATH}: build it first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C "
            "deep-successor-features-for-transfer_amd/csrc)")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib.sfx_last_error().decode(errors="replace")
        raise SFXError(f"{what or 'libsfx'} failed (status {rc}): {msg}")


def version() -> str:
    return lib.sfx_version().decode()


def fptr(arr) -> "C.POINTER(C.c_float)":
    """Host float32 numpy array -> float*."""
    return arr.ctypes.data_as(_FP)


def dptr(t) -> int:
    """Device tensor (or None) -> raw device pointer for *_dev arguments."""
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device_index: int) -> int:
    """The hipStream_t of torch's current stream on a device (per call: a `with torch.cuda.stream`
    block changes it).  torch.cuda.current_stream(dev).cuda_stream costs ≈7 µs of device-argument
    parsing per call on the drop-in's per-step path; the raw accessor returns the same pointer."""
    if _raw_stream is not None:
        return _raw_stream(device_index)
    return torch.cuda.current_stream(device_index).cuda_stream


class HostBuffer:
    """Coherent, device-mapped host memory (sfx_host_alloc): kernels read it directly.  `.np` is a
    numpy int64 view of `n` words; `.ptr` the address (the same on host and device)."""

    def __init__(self, n: int):
        import numpy as np

        p = C.c_void_p()
        check(lib.sfx_host_alloc(8 * int(n), C.byref(p)), "sfx_host_alloc")
        self.ptr = p.value
        self.np = np.ctypeslib.as_array((C.c_int64 * int(n)).from_address(self.ptr))

    def __del__(self):
        p, self.ptr = getattr(self, "ptr", None), None
        if p:
            try:
                lib.sfx_host_free(p)
            except Exception:
                pass
