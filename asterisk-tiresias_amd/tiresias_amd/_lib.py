"""ctypes binding of lib/libtiresias_fp.so (include/tiresias_fp.h).

The shared library is the product: every fingerprint and every search runs in its gfx950
kernels. There is no Python or CPU fallback — if the library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TFP_LIB_PATH: another build of the same library (kernel A/B experiments, scripts/ab_libs.sh)
LIB_PATH = os.environ.get("TFP_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libtiresias_fp.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "tiresias_fp.h")

TFP_OK = 0
ERRORS = {-1: "TFP_E_ARG", -2: "TFP_E_HIP", -3: "TFP_E_NOMEM", -4: "TFP_E_NOENT", -5: "TFP_E_CAPACITY",
          -6: "TFP_E_EXISTS", -7: "TFP_E_NODEV", -8: "TFP_E_FORMAT"}
NULL_MICRO = -(2**31)


class TfpError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Frame(C.Structure):
    _fields_ = [("frame_idx", C.c_int32), ("m1", C.c_int32), ("m2", C.c_int32), ("reserved", C.c_int32),
                ("q1", C.c_double), ("q2", C.c_double)]


class SearchParams(C.Structure):
    _fields_ = [("coefs", C.c_int32), ("freq_ignore_low", C.c_int32), ("freq_ignore_high", C.c_int32),
                ("reserved", C.c_int32), ("tolerance", C.c_double)]


class Result(C.Structure):
    _fields_ = [("found", C.c_int32), ("match_count", C.c_int32), ("frame_count", C.c_int32),
                ("clip_id", C.c_int32), ("uuid", C.c_char * 64)]


class SynthSpec(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("clip", C.c_int64), ("offset", C.c_int64)]


P = C.c_void_p
_SIGS = {
    "tfp_abi_version": (C.c_int, []),
    "tfp_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
    "tfp_engine_create": (C.c_int, [C.c_int32, C.POINTER(P)]),
    "tfp_engine_destroy": (None, [P]),
    "tfp_engine_last_error": (C.c_char_p, [P]),
    "tfp_frame_count": (C.c_int64, [C.c_int64]),
    "tfp_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(P)]),
    "tfp_host_free": (None, [P]),
    "tfp_wav_decode": (C.c_int, [P, C.c_int64, P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_wav_read": (C.c_int, [C.c_char_p, P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_wav_decode_f32": (C.c_int, [P, C.c_int64, P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_wav_read_f32": (C.c_int, [C.c_char_p, P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_fingerprint_f32_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_search_f32_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_fingerprint_pcm": (C.c_int, [P, P, C.c_int64, C.c_int32, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_fingerprint_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_plan_create": (C.c_int, [P, P, C.c_int32, C.c_int32, C.POINTER(P)]),
    "tfp_plan_destroy": (None, [P]),
    "tfp_plan_frames": (C.c_int64, [P]),
    "tfp_fingerprint_device": (C.c_int, [P, P, P, P, P, P]),
    "tfp_index_add": (C.c_int, [P, C.c_char_p, P, P, C.c_int32, C.POINTER(C.c_int32)]),
    "tfp_index_add_device": (C.c_int, [P, C.c_int32, C.POINTER(C.c_char_p), P, P, P]),
    "tfp_index_add_batch": (C.c_int, [P, C.c_int32, C.POINTER(C.c_char_p), P, P, P]),
    "tfp_index_rows": (C.c_int, [P, C.c_char_p, P, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_index_remove": (C.c_int, [P, C.c_char_p]),
    "tfp_index_clear": (C.c_int, [P]),
    "tfp_index_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_index_commit": (C.c_int, [P]),
    "tfp_index_build_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "tfp_index_set_tiebreak": (C.c_int, [P, P, C.c_int32]),
    "tfp_index_update_tiebreak": (C.c_int, [P, C.c_int32, P, C.c_int32]),
    "tfp_index_delta_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_search": (C.c_int, [P, P, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_search_batch": (C.c_int, [P, P, P, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_search_pcm_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_search_pcm_gather": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_search_coalesce_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "tfp_search_device": (C.c_int, [P, P, P, C.POINTER(SearchParams), P, P]),
    "tfp_search_q_device": (C.c_int, [P, P, P, C.c_int32, C.POINTER(SearchParams), P, P]),
    "tfp_index_uuid_of_key": (C.c_int, [P, C.c_int32, C.c_char_p, C.c_int32]),
    "tfp_stream_create": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int64, C.POINTER(P)]),
    "tfp_stream_destroy": (None, [P]),
    "tfp_stream_reset": (C.c_int, [P, C.c_int32]),
    "tfp_stream_push": (C.c_int, [P, P, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_synth_pcm": (C.c_int, [P, C.c_int32, C.c_int64, P]),
    "tfp_synth_pcm_device": (C.c_int, [P, P, C.c_int32, C.c_int64, P, P]),
    "tfp_synchronize": (C.c_int, [P, P]),
    "tfp_group_create": (C.c_int, [P, C.c_int32, C.POINTER(P)]),
    "tfp_group_destroy": (None, [P]),
    "tfp_index_cache_stats": (C.c_int, [P] + [C.POINTER(C.c_int64)] * 7),
    "tfp_sweep_stats": (C.c_int, [P] + [C.POINTER(C.c_int64)] * 4),
    "tfp_group_size": (C.c_int32, [P]),
    "tfp_group_tiebreak_stats": (C.c_int, [P] + [C.POINTER(C.c_int64)] * 3),
    "tfp_group_peer_stats": (C.c_int, [P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "tfp_group_last_error": (C.c_char_p, [P]),
    "tfp_group_engine": (P, [P, C.c_int32]),
    "tfp_group_fingerprint_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_group_fingerprint_f32_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_group_index_add": (C.c_int, [P, C.c_char_p, P, P, C.c_int32]),
    "tfp_group_index_add_batch": (C.c_int, [P, C.c_int32, C.POINTER(C.c_char_p), P, P, P]),
    "tfp_group_index_remove": (C.c_int, [P, C.c_char_p]),
    "tfp_group_index_clear": (C.c_int, [P]),
    "tfp_group_index_rows": (C.c_int, [P, C.c_char_p, P, P, C.c_int64, C.POINTER(C.c_int64)]),
    "tfp_group_index_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "tfp_group_index_commit": (C.c_int, [P]),
    "tfp_group_search_batch": (C.c_int, [P, P, P, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_group_search_pcm_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_group_search_f32_batch": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_group_search_pcm_gather": (C.c_int, [P, P, P, C.c_int32, C.c_int32, C.POINTER(SearchParams), P]),
    "tfp_group_search_coalesce_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "tfp_group_stream_create": (C.c_int, [P, C.c_int32, C.c_int32, C.c_int64, C.POINTER(P)]),
    "tfp_group_stream_destroy": (None, [P]),
    "tfp_group_stream_reset": (C.c_int, [P, C.c_int32]),
    "tfp_group_stream_push": (C.c_int, [P, P, C.c_int32, C.POINTER(SearchParams), P]),
}

_lib = None


def header_symbols() -> list[str]:
    """Every function the C-ABI header declares."""
    with open(HEADER) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**(tfp_[a-z_0-9]+)\s*\(", src, re.M)))


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                              "(the HIP engine is the only implementation; there is no fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("TFP_LIB_PATH") and not hasattr(L, name):
                continue  # an older A/B build without this entry point (calling it raises AttributeError)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, eng=None):
    """Raise TfpError for a non-OK code; eng None reads the thread's engine-less error."""
    if rc != TFP_OK:
        raise TfpError(rc, lib().tfp_engine_last_error(eng).decode())
    return rc
