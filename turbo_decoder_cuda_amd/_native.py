"""ctypes binding of libturbo_mi355x.so (the C ABI in include/turbo_mi355x.h).

The library is built in-tree by turbo_decoder_cuda_amd/build.py.  There is no fallback: if
the shared object is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TD_LIB_PATH") or os.path.join(PKG, "libturbo_mi355x.so")

TD_OK, TD_EINVAL, TD_ENOMEM, TD_EHIP, TD_ENODEV = 0, 1, 2, 3, 4
TD_ALGO_LOGMAP, TD_ALGO_MAXLOG = 0, 1
TD_F64, TD_F32 = 0, 1
TD_WMAXSTAR_FAST, TD_WMAXSTAR_EXACT = 0, 1
TD_MAXSTAR_WINDOW_FAST = 2   # td_maxstar_host_* algo: the windowed one-read table

# every symbol include/turbo_mi355x.h declares (tests check the .so exports all of them)
EXPORTS = (
    "td_create", "td_destroy", "td_reserve", "td_decode_device", "td_decode_host", "td_siso_host",
    "td_last_error", "td_device_count", "td_abi_version", "td_maxstar_host_f64", "td_maxstar_host_f32",
    "td_trellis_tables", "td_qpp_table", "td_profile_enable", "td_profile_read", "td_debug_set_stamps",
    "td_debug_stamp_slots", "td_synth_seed", "td_synth_frames", "td_count_errors", "td_rand_window", "td_synth_seek",
    "td_set_window", "td_synth_modulation", "td_modulate", "td_demodulate", "td_debug_placement",
    "td_debug_placement_rule", "td_clock_read", "td_window_steps", "td_debug_placement_cost", "td_debug_window_layout",
    "td_debug_workspace_bytes", "td_set_window_maxstar",
)


class TdParams(C.Structure):
    _fields_ = [
        ("K", C.c_int), ("f1", C.c_int), ("f2", C.c_int), ("iterations", C.c_int),
        ("algo", C.c_int), ("precision", C.c_int), ("device", C.c_int),
    ]


class TdWindowParams(C.Structure):
    _fields_ = [("window", C.c_int), ("overlap", C.c_int), ("nii", C.c_int), ("concurrent", C.c_int),
                ("ext_scale", C.c_double)]


class TurboError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"turbo_mi355x error {code}: {msg}")
        self.code = code


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -m turbo_decoder_cuda_amd.build` "
            "(there is no CPU fallback)")
    try:   # torch ships its own libamdhip64.so.7 (same soname): load it first so the library and
        import torch  # noqa: F401  torch bind to one HIP runtime (the other order hides the GPUs from torch)
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P, I = C.c_void_p, C.c_int
    L.td_create.argtypes = [C.POINTER(P), C.POINTER(TdParams)]
    L.td_destroy.argtypes = [P]
    L.td_reserve.argtypes = [P, I]
    L.td_decode_device.argtypes = [P, P, I, P, I, P, P]
    L.td_decode_host.argtypes = [P, P, I, P, P]
    L.td_siso_host.argtypes = [P, P, P, I, P, I, I]
    L.td_last_error.restype = C.c_char_p
    L.td_device_count.restype = I
    L.td_abi_version.restype = I
    L.td_maxstar_host_f64.argtypes = [C.c_double, C.c_double, I]
    L.td_maxstar_host_f64.restype = C.c_double
    L.td_maxstar_host_f32.argtypes = [C.c_float, C.c_float, I]
    L.td_maxstar_host_f32.restype = C.c_float
    L.td_trellis_tables.argtypes = [P, P, P]
    L.td_qpp_table.argtypes = [I, I, I, P]
    L.td_profile_enable.argtypes = [P, I]
    L.td_debug_set_stamps.argtypes = [P, P]
    L.td_debug_stamp_slots.restype = I
    L.td_debug_placement.argtypes = [P, C.POINTER(C.c_float), I, C.POINTER(C.c_int)]
    L.td_debug_placement_rule.argtypes = [C.POINTER(C.c_float), I]
    if hasattr(L, "td_debug_placement_cost"):   # (older A/B builds loaded by TD_LIB_PATH lack it)
        L.td_debug_placement_cost.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.td_profile_read.argtypes = [P, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_int)]
    if hasattr(L, "td_clock_read"):   # measurement support (older A/B builds loaded by TD_LIB_PATH lack it)
        L.td_clock_read.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.td_synth_seed.argtypes = [P, C.c_uint]
    L.td_rand_window.argtypes = [C.c_uint, C.c_ulonglong, P]
    L.td_synth_seek.argtypes = [P, C.c_ulonglong]
    L.td_synth_frames.argtypes = [P, C.c_double, I, P, P, P]
    L.td_count_errors.argtypes = [P, P, I, P, I, P, P]
    L.td_set_window.argtypes = [P, C.POINTER(TdWindowParams)]
    L.td_synth_modulation.argtypes = [P, I]
    L.td_modulate.argtypes = [P, C.c_longlong, I, P, P, P]
    L.td_demodulate.argtypes = [P, P, C.c_longlong, I, C.c_double, P, P]
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != TD_OK:
        raise TurboError(rc, lib().td_last_error().decode(errors="replace"))
