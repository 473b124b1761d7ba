"""HIP streams that each get a hardware queue of their own, for running several codec handles side by side.

The HIP runtime maps every stream a process creates onto one of GPU_MAX_HW_QUEUES hardware queues (default 4);
two busy streams that share a queue run one after the other.  torch's stream pool hands out streams whose
queues collide (measured on MI355X, tools/decN_exp.py, 32 x 384x384 raster decodes side by side: 4 decodes on
pool streams 1.81x the throughput of one, on streams created here 2.90x).  Streams created consecutively here,
before any other stream is busy, land on distinct queues as long as the process has enough of them
(GPU_MAX_HW_QUEUES >= busy streams + 1 for the null stream; bench.py sets it before HIP starts).
"""
from __future__ import annotations

import ctypes
from typing import List

import torch

_hip = None


def _runtime():
    """The HIP runtime torch has loaded (one runtime per process: load it by its mapped path)."""
    global _hip
    if _hip is None:
        torch.cuda.init()
        path = None
        with open("/proc/self/maps") as fh:
            for line in fh:
                if "libamdhip64" in line:
                    path = line.split()[-1]
                    break
        _hip = ctypes.CDLL(path or "libamdhip64.so")
        _hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        _hip.hipStreamCreateWithFlags.restype = ctypes.c_int
        _hip.hipSetDevice.argtypes = [ctypes.c_int]
        _hip.hipSetDevice.restype = ctypes.c_int
        _hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    return _hip


def cu_mask(fraction: float, n_cu: int) -> List[int]:
    """32-bit words of a CU mask selecting round(fraction * n_cu) CUs spread evenly over the CU index range (so every
    XCD / shader engine keeps its share whatever the index -> CU mapping)."""
    k = max(1, min(n_cu, int(round(fraction * n_cu))))
    bits = [False] * n_cu
    for i in range(k):
        bits[(i * n_cu) // k] = True
    words = [0] * ((n_cu + 31) // 32)
    for i, b in enumerate(bits):
        if b:
            words[i // 32] |= 1 << (i % 32)
    return words


def dedicated_streams(n: int, device: torch.device, masks=None) -> List[torch.cuda.ExternalStream]:
    """n non-blocking HIP streams on `device`, created back to back (hipStreamCreateWithFlags; stream i with
    hipExtStreamCreateWithCUMask when masks[i] is a list of mask words, see cu_mask), wrapped as torch external
    streams.  They live for the rest of the process."""
    hip = _runtime()
    if hip.hipSetDevice(device.index or 0) != 0:
        raise RuntimeError("hipSetDevice failed")
    out = []
    for i in range(n):
        s = ctypes.c_void_p()
        mk = masks[i] if masks else None
        if mk:
            arr = (ctypes.c_uint32 * len(mk))(*mk)
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(mk), arr)
        else:
            rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)      # hipStreamNonBlocking
        if rc != 0:
            raise RuntimeError(f"stream creation failed ({rc})")
        out.append(torch.cuda.ExternalStream(s.value, device=device))
    return out
