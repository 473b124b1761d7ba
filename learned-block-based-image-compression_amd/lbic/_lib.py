"""ctypes binding of liblbic.so (include/lbic.h).  Fails loudly: there is no CPU fallback.

The library is built in-tree (``make -C csrc``, or ``__graft_entry__.build()``) so it travels with
the repository snapshot to the GPU box.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblbic.so")
if os.environ.get("LBIC_LIB_VARIANT"):      # A/B experiments: lbic/liblbic_<variant>.so built from another revision
    LIB_PATH = os.path.join(HERE, f"liblbic_{os.environ['LBIC_LIB_VARIANT']}.so")

LBC_E_NOT_UPDATED = -4


class LbcKernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 40), ("launches", ctypes.c_longlong), ("total_launches", ctypes.c_longlong),
                ("total_ms", ctypes.c_double),
                ("flops", ctypes.c_double), ("bytes", ctypes.c_double),
                ("launches_chain", ctypes.c_longlong), ("total_ms_chain", ctypes.c_double),
                ("total_flops", ctypes.c_double), ("total_bytes", ctypes.c_double)]


class LbcConfig(ctypes.Structure):
    _fields_ = [("block_size", ctypes.c_int), ("ks", ctypes.c_int * 4), ("n", ctypes.c_int),
                ("m", ctypes.c_int), ("device", ctypes.c_int)]


_P = ctypes.c_void_p
_SIGS = {
    "lbc_create": ([ctypes.POINTER(LbcConfig), ctypes.POINTER(_P)], ctypes.c_int),
    "lbc_destroy": ([_P], None),
    "lbc_create_sibling": ([_P, ctypes.POINTER(_P)], ctypes.c_int),
    "lbc_set_tensor": ([_P, ctypes.c_char_p, _P, ctypes.POINTER(ctypes.c_int64), ctypes.c_int], ctypes.c_int),
    "lbc_finalize": ([_P], ctypes.c_int),
    "lbc_pmf_to_quantized_cdf": ([_P, ctypes.c_int, ctypes.c_int, _P], ctypes.c_int),
    "lbc_set_entropy_tables": ([_P, _P, ctypes.c_int, _P, ctypes.c_int, _P, _P], ctypes.c_int),
    "lbc_encode": ([_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, _P], ctypes.c_int),
    "lbc_rans_encode": ([_P, _P, _P, ctypes.c_size_t, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t)],
                        ctypes.c_int),
    "lbc_rans_decode_host": ([_P, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "lbc_rans_decode_gpu": ([_P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, _P,
                             ctypes.c_int, _P, _P], ctypes.c_int),
    "lbc_decode": ([_P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, ctypes.c_int,
                    ctypes.c_int, _P, _P], ctypes.c_int),
    "lbc_decode_team": ([ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t),
                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P), _P], ctypes.c_int),
    "lbc_team_stamps": ([_P, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
                        ctypes.c_int),
    "lbc_team_mode": ([_P, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "lbc_team_events": ([_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "lbc_decode_path": ([_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "lbc_one_stamps": ([_P, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
                       ctypes.c_int),
    "lbc_team_stats": ([_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "lbc_encode_ex": ([_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P, ctypes.c_int, _P],
                      ctypes.c_int),
    "lbc_set_option": ([_P, ctypes.c_int, ctypes.c_longlong], ctypes.c_int),
    "lbc_forward": ([_P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P], ctypes.c_int),
    "lbc_rans_encode_rows": ([_P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P),
                              ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "lbc_decode_rows": ([_P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int, ctypes.c_int,
                         ctypes.c_int, _P, _P], ctypes.c_int),
    "lbc_band_begin": ([_P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P], ctypes.c_int),
    "lbc_band_run": ([_P, ctypes.c_int, ctypes.c_int, _P, _P, _P], ctypes.c_int),
    "lbc_band_end": ([_P, _P, _P, _P, _P, _P], ctypes.c_int),
    "lbc_free": ([_P], None),
    "lbc_last_error": ([], ctypes.c_char_p),
    "lbc_last_timing": ([_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
    "lbc_profile_begin": ([_P, ctypes.c_int], ctypes.c_int),
    "lbc_profile_end": ([_P, ctypes.POINTER(LbcKernelStat), ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
                        ctypes.c_int),
}
EXPORTS = tuple(_SIGS)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"liblbic.so not built ({LIB_PATH}); run __graft_entry__.build() or make -C csrc")
        lb = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lb, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lb
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().lbc_last_error().decode(errors="replace")
        if rc == LBC_E_NOT_UPDATED:
            raise ValueError(msg)
        raise RuntimeError(f"liblbic error {rc}: {msg}")
    return rc


def ptr(t):
    """Raw pointer of a contiguous torch tensor or numpy array."""
    if hasattr(t, "data_ptr"):
        return ctypes.c_void_p(t.data_ptr())
    return t.ctypes.data_as(ctypes.c_void_p)
