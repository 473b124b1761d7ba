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
        _hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                      ctypes.POINTER(ctypes.c_uint32)]
        _hip.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
        _hip.hipSetDevice.argtypes = [ctypes.c_int]
        _hip.hipSetDevice.restype = ctypes.c_int
    return _hip


def dedicated_streams(n: int, device: torch.device) -> List[torch.cuda.ExternalStream]:
    """n non-blocking HIP streams on `device`, created back to back (hipStreamCreateWithFlags), wrapped as torch
    external streams.  They live for the rest of the process."""
    hip = _runtime()
    if hip.hipSetDevice(device.index or 0) != 0:
        raise RuntimeError("hipSetDevice failed")
    out = []
    for _ in range(n):
        s = ctypes.c_void_p()
        rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), 1)      # hipStreamNonBlocking
        if rc != 0:
            raise RuntimeError(f"stream creation failed ({rc})")
        out.append(torch.cuda.ExternalStream(s.value, device=device))
    return out


def xcd_slot_mask(cus: int, slots) -> List[int]:
    """CU mask (32-bit words) of the CU slots `slots` (0 .. cus/8 - 1) on EVERY XCD.  Bit i of a
    hipExtStreamCreateWithCUMask mask is CU slot i // 8 of XCD i % 8 on MI355X, and slot j lies on shader engine j % 4
    (csrc/cumask_probe.hip, profiles/r03_exp/r03_cumask_probe.txt)."""
    per = cus // 8
    if cus % 8 or any(not 0 <= j < per for j in slots):
        raise ValueError(f"bad CU slots for {cus} CUs")
    words = [0] * ((cus + 31) // 32)
    for i in range(cus):
        if i // 8 in slots:
            words[i // 32] |= 1 << (i % 32)
    return words


def cu_masked_stream(words: List[int], device: torch.device) -> torch.cuda.ExternalStream:
    """A non-blocking HIP stream whose kernels run only on the CUs of `words` (hipExtStreamCreateWithCUMask: a
    hardware queue of its own with that CU mask).  It lives for the rest of the process."""
    hip = _runtime()
    if hip.hipSetDevice(device.index or 0) != 0:
        raise RuntimeError("hipSetDevice failed")
    s = ctypes.c_void_p()
    arr = (ctypes.c_uint32 * len(words))(*words)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), arr)
    if rc != 0:
        raise RuntimeError(f"CU-masked stream creation failed ({rc})")
    return torch.cuda.ExternalStream(s.value, device=device)


def split_slots(per: int, dec: int):
    """(decoder slots, encoder slots) of one XCD: the decoder takes shader engine 0's slots first, then engine 1's ...
    (slot order by (j % 4, j // 4)), so for 8 <= dec <= per - 8 both sides hold a slot of every group of four
    consecutive slots -- every XCD keeps CUs on both sides whichever way the mask's bits map onto XCDs."""
    order = sorted(range(per), key=lambda j: (j % 4, j // 4))
    return set(order[:dec]), set(order[dec:])


def cu_split_streams(dec_slots: int, device: torch.device):
    """(encoder stream, decoder stream) on disjoint CUs: the decoder on `dec_slots` CUs of every XCD, the encoder on
    the rest."""
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    per = cus // 8
    if not 8 <= dec_slots <= per - 8:
        raise ValueError(f"decoder CUs per XCD must be in [8, {per - 8}]")
    dec, enc = split_slots(per, dec_slots)
    return cu_masked_stream(xcd_slot_mask(cus, enc), device), cu_masked_stream(xcd_slot_mask(cus, dec), device)
