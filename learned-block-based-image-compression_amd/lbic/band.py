"""Band pipeline: one batch of frames split over the ranks of a process group by block rows.

Rank p codes block rows [v0_p, v0_p + rows_p) of every frame with compress() semantics (lbc_band_*).  The frames'
anti-diagonal wavefront codes block (v, h) at global step t = h + 2v; ranks run the global steps in chunks of
`chunk`, each rank one chunk behind the rank above: before chunk c it receives the two block rows above its band
from rank p-1 (which has run chunk c), and after it sends its own last two rows to rank p+1 -- one point-to-point
hand-off of 2 x Wb x 3B^2 floats per image and chunk.  Results are bit-identical to coding the whole frame on one
GPU (tests/test_band_gpu.py); the bands' symbols concatenated in row order are the frame's, so rank 0 can write
the reference bitstream.

This is the only way to spread ONE frame over GPUs; it does not shorten the wavefront (its critical path is
(Wb-1) + 2(Hb-1) + 1 steps on any number of GPUs plus one chunk per extra rank), it divides the work per step:
worth it only for frames whose wavefront steps are throughput-bound on one GPU.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch

from . import _lib


def band_rows(Hb: int, parts: int) -> List[Tuple[int, int]]:
    """[(v0, rows)] of `parts` contiguous bands covering Hb block rows (the first Hb % parts bands one row taller)."""
    if parts < 1 or parts > Hb:
        raise ValueError(f"cannot split {Hb} block rows into {parts} bands")
    base, extra = divmod(Hb, parts)
    out, v0 = [], 0
    for p in range(parts):
        r = base + (1 if p < extra else 0)
        out.append((v0, r))
        v0 += r
    return out


def wavefront_steps(Hb: int, Wb: int) -> int:
    return (Wb - 1) + 2 * (Hb - 1) + 1


def compress_band(model, xb_band: torch.Tensor, v0: int, Hb: int, group=None, chunk: int = 16,
                  transport: str = "device") -> dict:
    """Code this rank's band of a batch of frames.  xb_band: [n, rows, Wb, 3B^2] fp32 on the model's device, rows
    [v0, v0 + rows) of frames Hb block rows tall; every rank of `group` calls this with its own band, ranks ordered
    top to bottom.  transport "device" sends device tensors (RCCL), "host" stages them through the CPU (gloo).
    Returns dict(zhat, symbols, indexes) of the band (device tensors)."""
    import torch.distributed as dist
    model._check_ready()
    rank = dist.get_rank(group) if group is not None or dist.is_initialized() else 0
    world = dist.get_world_size(group) if group is not None or dist.is_initialized() else 1
    n, rows, Wb, C = xb_band.shape
    if C != model.arch.cx or xb_band.device != model.device or xb_band.dtype != torch.float32:
        raise ValueError("xb_band must be [n, rows, Wb, 3B^2] float32 on the model's device")
    xb_band = xb_band.contiguous()
    L = _lib.lib()
    stream = torch.cuda.current_stream(model.device)
    sp = ctypes.c_void_p(stream.cuda_stream)
    _lib.check(L.lbc_band_begin(model._h, _lib.ptr(xb_band), n, rows, Wb, v0, sp))
    halo = torch.zeros((n, 2, Wb, C), dtype=torch.float32, device=model.device) if rank > 0 else None
    edge = torch.empty((n, 2, Wb, C), dtype=torch.float32, device=model.device) if rank < world - 1 else None
    prev_rank = None if rank == 0 else _global(rank - 1, group)
    next_rank = None if rank == world - 1 else _global(rank + 1, group)
    T = wavefront_steps(Hb, Wb)
    for t0 in range(0, T, chunk):
        t1 = min(T, t0 + chunk)
        if halo is not None:                     # rank p-1 has run [t0, t1): its last rows cover what we read
            _recv(halo, prev_rank, group, transport, stream)
        _lib.check(L.lbc_band_run(model._h, t0, t1, _lib.ptr(halo) if halo is not None else None,
                                  _lib.ptr(edge) if edge is not None else None, sp))
        if edge is not None:
            _send(edge, next_rank, group, transport, stream)
    zhat = torch.empty_like(xb_band)
    nsym = rows * Wb * model.arch.M
    sym = torch.empty((n, nsym), dtype=torch.int32, device=model.device)
    idx = torch.empty((n, nsym), dtype=torch.int32, device=model.device)
    _lib.check(L.lbc_band_end(model._h, _lib.ptr(zhat), _lib.ptr(sym), _lib.ptr(idx), None, sp))
    return dict(zhat=zhat, symbols=sym, indexes=idx)


def gather_bands(part: dict, group=None, dst: int = 0) -> Optional[dict]:
    """All bands' zhat / symbols / indexes concatenated in row order on rank `dst` (None elsewhere).  Bands may differ
    in height, so the row counts are all-gathered first.  Tensors travel on the device with RCCL, through the host
    with gloo."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    host = dist.get_backend(group) == "gloo"
    z, s, i = (part[k].cpu() if host else part[k] for k in ("zhat", "symbols", "indexes"))
    rows = torch.tensor([z.shape[1]], dtype=torch.int64, device=z.device)
    allrows = [torch.zeros_like(rows) for _ in range(world)]
    dist.all_gather(allrows, rows, group=group)
    if rank != dst:
        for t in (z, s, i):
            dist.send(t.contiguous(), _global(dst, group), group=group)
        return None
    zs, ss, is_ = [], [], []
    n, _, Wb, C = z.shape
    M = s.shape[1] // (z.shape[1] * Wb)
    for p in range(world):
        r = int(allrows[p])
        if p == dst:
            zp, sp_, ip = z, s, i
        else:
            zp = torch.empty((n, r, Wb, C), dtype=z.dtype, device=z.device)
            sp_ = torch.empty((n, r * Wb * M), dtype=s.dtype, device=z.device)
            ip = torch.empty((n, r * Wb * M), dtype=i.dtype, device=z.device)
            for t in (zp, sp_, ip):
                dist.recv(t, _global(p, group), group=group)
        zs.append(zp)
        ss.append(sp_)
        is_.append(ip)
    return dict(zhat=torch.cat(zs, 1), symbols=torch.cat(ss, 1), indexes=torch.cat(is_, 1))


def _global(r, group):
    import torch.distributed as dist
    return r if group is None else dist.get_global_rank(group, r)


def _send(t, dst, group, transport, stream):
    import torch.distributed as dist
    if transport == "host":
        stream.synchronize()
        dist.send(t.cpu(), dst, group=group)
    else:
        dist.send(t, dst, group=group)


def _recv(t, src, group, transport, stream):
    import torch.distributed as dist
    if transport == "host":
        h = torch.empty(t.shape, dtype=t.dtype)
        dist.recv(h, src, group=group)
        t.copy_(h)
    else:
        dist.recv(t, src, group=group)
