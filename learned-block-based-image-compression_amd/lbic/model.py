"""``BlockBasedImgCompLossyNetv9`` -- the reference's model interface over liblbic.so.

Mirrors graphs/models/BlockBasedImgCompLossy_net.py:251-452: the same constructor argument (the
config), ``load_state_dict`` with the reference's keys, ``update(force)``, ``compress(x, LRU, chlat)``
-> (bitstream, zhat) and ``decompress(bitstream, LRU, xshape, chlat, devc)`` -> zhat, on the same NCHW
block->channel tensors [1, 3B^2, H/B, W/B].  The arithmetic runs in HIP kernels; there is no CPU path.
``compress_batch`` / ``decompress_batch`` add the batched form used by bench.py (BASELINE config 2:
a batch of 32 frames on one GPU) on block-major [n, Hb, Wb, 3B^2] device tensors.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Sequence

import numpy as np
import torch

from . import _lib
from .arch import Arch, arch_from_config
from .entropy import GaussianConditional, get_scale_table


class BlockBasedImgCompLossyNetv9:
    def __init__(self, config, device=None):
        self.config = config
        self.arch: Arch = arch_from_config(config)
        if self.arch.KS[0] != 3:
            raise ValueError("KS[0] must be 3 (all reference configs)")
        if device is None:
            device = torch.device("cuda", int(getattr(config, "gpu_device", 0) or 0))
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("BlockBasedImgCompLossyNetv9 runs on the GPU only (HIP kernels, no CPU path)")
        self.conditional_gaussian_model = GaussianConditional()
        self._params: Dict[str, torch.Tensor] = {}
        cfg = _lib.LbcConfig()
        cfg.block_size = self.arch.B
        for i, k in enumerate(self.arch.KS):
            cfg.ks[i] = k
        cfg.n, cfg.m = self.arch.N, self.arch.M
        cfg.device = self.device.index or 0
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().lbc_create(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h
        self._tables_uploaded = False
        self.training = False
        self._pool = None
        self._pool_workers = 0

    def sibling(self) -> "BlockBasedImgCompLossyNetv9":
        """Another model object on the same loaded weights (lbc_create_sibling): the packed device weights are
        shared, the workspaces, graphs and device entropy tables are its own, so it can code on another stream
        from another thread while this one is busy (bench.py's decode passes).  Needs load_state_dict() first;
        the CDFs are those of this object at the time of the call."""
        if not self._params:
            raise RuntimeError("load_state_dict() before sibling()")
        m = BlockBasedImgCompLossyNetv9.__new__(BlockBasedImgCompLossyNetv9)
        m.config, m.arch, m.device = self.config, self.arch, self.device
        m.conditional_gaussian_model = self.conditional_gaussian_model
        m._params = self._params
        m.training = False
        m._pool = None
        m._pool_workers = 0
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().lbc_create_sibling(self._h, ctypes.byref(h)))
        m._h = h
        m._tables_uploaded = self._tables_uploaded
        if self._tables_uploaded:
            m._keep = self._keep
        return m

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib().lbc_destroy(h)
            except Exception:
                pass
            self._h = None

    # ------------------------------------------------------------------ nn.Module-like surface
    def eval(self):
        self.training = False
        return self

    def to(self, device):
        if torch.device(device) != self.device:
            raise RuntimeError("device is fixed at construction (one handle per GPU)")
        return self

    def parameters(self):
        return iter(self._params.values())

    def state_dict(self):
        sd = dict(self._params)
        sd.update(self.conditional_gaussian_model.state_dict())
        return sd

    def load_state_dict(self, sd, strict: bool = True):
        """Reference keys (arch.param_shapes); buffers (mask, pedestal, bound) are accepted."""
        names = {n for n, _ in self.arch.param_shapes()}
        missing = [n for n in names if n not in sd]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}...")
        L = _lib.lib()
        for k, v in sd.items():
            if k.startswith("conditional_gaussian_model."):
                continue
            t = torch.as_tensor(np.asarray(v) if not torch.is_tensor(v) else v).detach().float().cpu().contiguous()
            if k in names:
                self._params[k] = t
            shape = (ctypes.c_int64 * t.dim())(*t.shape)
            _lib.check(L.lbc_set_tensor(self._h, k.encode(), _lib.ptr(t), shape, t.dim()))
        _lib.check(L.lbc_finalize(self._h))
        return self

    # ------------------------------------------------------------------ entropy model
    def update(self, force=False):
        """net:121-125: build the scale table and the quantized CDFs; pushes them to the device."""
        updated = self.conditional_gaussian_model.update_scale_table(get_scale_table(), force=force)
        if updated or not self._tables_uploaded:
            self._upload_tables()
        return updated

    def _upload_tables(self):
        gc = self.conditional_gaussian_model
        gc._check_cdf_size()
        gc._check_cdf_length()
        gc._check_offsets_size()
        table = gc.scale_table.float().contiguous().numpy()
        cdf = gc.quantized_cdf.int().contiguous().numpy()
        ln = gc.cdf_length.int().contiguous().numpy()
        off = gc.offset.int().contiguous().numpy()
        _lib.check(_lib.lib().lbc_set_entropy_tables(self._h, _lib.ptr(table), len(table), _lib.ptr(cdf),
                                                     cdf.shape[1], _lib.ptr(ln), _lib.ptr(off)))
        self._keep = (table, cdf, ln, off)
        self._tables_uploaded = True

    def _check_ready(self):
        gc = self.conditional_gaussian_model
        gc._check_cdf_size()
        gc._check_cdf_length()
        gc._check_offsets_size()
        if not self._tables_uploaded:
            self._upload_tables()

    def _check_lru(self, LRU):
        if LRU is not None and tuple(int(v) for v in LRU) != (self.arch.lru,) * 3:
            raise ValueError(f"LRU {list(LRU)} != compress/decompress receptive field {[self.arch.lru] * 3} "
                             "(agents/blkbsdimgcomp_agent.py:481-489)")

    # ------------------------------------------------------------------ batched GPU path
    def compress_batch(self, xb: torch.Tensor, want_bits: bool = False, frame_pad: bool = False):
        """xb: [n, Hb, Wb, 3B^2] fp32 on this device.  Returns dict(streams, zhat, symbols, indexes, bits)
        with device tensors (symbols/indexes [n, Hb*Wb*M] int32, zhat like xb).  frame_pad: the closed loop of
        validate_recu_reco (forward()'s border rule); needs no CDFs (indexes are 0 before update())."""
        if not frame_pad:
            self._check_ready()
        elif self.conditional_gaussian_model._quantized_cdf.numel() and not self._tables_uploaded:
            self._upload_tables()
        if xb.device != self.device or xb.dtype != torch.float32 or xb.dim() != 4 or xb.shape[3] != self.arch.cx:
            raise ValueError("xb must be [n, Hb, Wb, 3B^2] float32 on the model's device")
        xb = xb.contiguous()
        n, Hb, Wb, _ = xb.shape
        zhat = torch.empty_like(xb)
        nsym = Hb * Wb * self.arch.M
        sym = torch.empty((n, nsym), dtype=torch.int32, device=self.device)
        idx = torch.empty((n, nsym), dtype=torch.int32, device=self.device)
        bits = torch.empty((n, nsym), dtype=torch.float32, device=self.device) if want_bits else None
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(_lib.lib().lbc_encode_ex(self._h, _lib.ptr(xb), n, Hb, Wb, _lib.ptr(zhat), _lib.ptr(sym),
                                            _lib.ptr(idx), _lib.ptr(bits) if bits is not None else None,
                                            1 if frame_pad else 0, ctypes.c_void_p(stream)))
        return dict(zhat=zhat, symbols=sym, indexes=idx, bits=bits)

    def entropy_encode(self, symbols: torch.Tensor, indexes: torch.Tensor, workers: int = 0, fmt: str = "reference",
                       Hb: int = 0, Wb: int = 0) -> List[bytes]:
        """BufferedRansEncoder per image (host C++), symbols/indexes [n, L] (any device).  fmt "reference":
        one stream per image as in the reference; fmt "rows": the opt-in sub-stream container (one stream per
        block row, lbc_rans_encode_rows; needs Hb, Wb).  Images are coded on parallel host threads
        (ctypes drops the GIL during the call)."""
        if fmt not in ("reference", "rows"):
            raise ValueError(f"unknown bitstream format {fmt!r}")
        s = symbols.to("cpu", torch.int32).contiguous().numpy()
        i = indexes.to("cpu", torch.int32).contiguous().numpy()
        L = _lib.lib()
        if fmt == "rows" and Hb * Wb * self.arch.M != s.shape[1]:
            raise ValueError("fmt='rows' needs the frame's Hb, Wb")

        def one(k):
            p = ctypes.c_void_p()
            ln = ctypes.c_size_t()
            if fmt == "rows":
                _lib.check(L.lbc_rans_encode_rows(self._h, _lib.ptr(s[k]), _lib.ptr(i[k]), Hb, Wb, ctypes.byref(p),
                                                  ctypes.byref(ln)))
            else:
                _lib.check(L.lbc_rans_encode(self._h, _lib.ptr(s[k]), _lib.ptr(i[k]), s.shape[1], ctypes.byref(p),
                                             ctypes.byref(ln)))
            b = ctypes.string_at(p, ln.value)
            L.lbc_free(p)
            return b

        n = s.shape[0]
        workers = workers or min(n, 16)
        if n == 1 or workers <= 1:
            return [one(k) for k in range(n)]
        if self._pool is None or self._pool_workers != workers:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=workers)
            self._pool_workers = workers
        return list(self._pool.map(one, range(n)))

    def decompress_batch(self, streams: Sequence[bytes], Hb: int, Wb: int, fmt: str = "reference") -> torch.Tensor:
        """Decode n bitstreams of Hb x Wb blocks on the GPU -> zhat [n, Hb, Wb, 3B^2].  fmt "reference": raster
        decode of one stream per image (the reference format); "rows": wavefront decode of the sub-stream
        containers of entropy_encode(fmt="rows")."""
        if fmt not in ("reference", "rows"):
            raise ValueError(f"unknown bitstream format {fmt!r}")
        self._check_ready()
        n = len(streams)
        # pointers into the callers' bytes objects (no copies); `bufs` keeps them alive during the call
        bufs = [s if isinstance(s, bytes) else bytes(s) for s in streams]
        arr = (ctypes.c_void_p * n)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in bufs])
        lens = (ctypes.c_size_t * n)(*[len(s) for s in streams])
        zhat = torch.empty((n, Hb, Wb, self.arch.cx), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        fn = _lib.lib().lbc_decode_rows if fmt == "rows" else _lib.lib().lbc_decode
        _lib.check(fn(self._h, arr, lens, n, Hb, Wb, _lib.ptr(zhat), ctypes.c_void_p(stream)))
        return zhat

    def team_stamps(self):
        """Raw stamps of the last decompress_teams launch led by this handle (LBIC_TEAM_STAMPS=1), [T, 256]
        (lbc_team_stamps, 256 per team): [op] after each barrier of the sampled raster step, [32 + op] rank 0's own
        work done, 60/61 the ends of the step before it and of the sampled step, 62/63 launch start / end (100 MHz);
        [256 + 64 op + p] shader-clock stamps inside the operation's GEMM (1024 words per team)."""
        L = _lib.lib()
        n = ctypes.c_int(0)
        _lib.check(L.lbc_team_stamps(self._h, None, 0, ctypes.byref(n)))
        buf = (ctypes.c_ulonglong * max(n.value, 1))()
        _lib.check(L.lbc_team_stamps(self._h, buf, n.value, ctypes.byref(n)))
        return [list(buf[i:i + 1024]) for i in range(0, n.value, 1024)]

    def team_stats(self):
        """The last decompress_teams launch led by this handle (lbc_team_stats): dict(launch_ms, bytes, flops,
        plain, mode, sc1_reruns, timeout_fallbacks) -- its duration, algorithmic bytes / FLOPs, the hand-off store mode
        it ran in, how the call decoded (lbc_team_mode: "team_sparse" / "team_dense" rANS variant, "fallback" to
        lbc_decode per batch, or for one batch of one image "one" / "graphs": lbc_decode's single-image decoder or its
        row graphs), and the handle's event counters (lbc_team_events): write-through reruns and barrier timeouts
        decoded through the fallback."""
        L = _lib.lib()
        ms, by, fl, pl = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        _lib.check(L.lbc_team_stats(self._h, ctypes.byref(ms), ctypes.byref(by), ctypes.byref(fl), ctypes.byref(pl)))
        mode = ctypes.c_int()
        _lib.check(L.lbc_team_mode(self._h, ctypes.byref(mode)))
        rr, to = ctypes.c_int(), ctypes.c_int()
        _lib.check(L.lbc_team_events(self._h, ctypes.byref(rr), ctypes.byref(to)))
        return dict(launch_ms=ms.value, bytes=by.value, flops=fl.value, plain=pl.value,
                    mode=("fallback", "team_sparse", "team_dense", "one", "graphs")[mode.value], sc1_reruns=rr.value,
                    timeout_fallbacks=to.value)

    def decode_path(self):
        """How the last decompress of this handle ran (lbc_decode_path): dict(path="graphs" | "one", one_timeouts) --
        "one" = the single-image persistent decoder k_dec_one (one image whose step weights fit the grid's LDS:
        B8_lowrate, B4_highrate)."""
        p, t = ctypes.c_int(), ctypes.c_int()
        _lib.check(_lib.lib().lbc_decode_path(self._h, ctypes.byref(p), ctypes.byref(t)))
        return dict(path=("graphs", "one")[p.value], one_timeouts=t.value)

    def one_stamps(self):
        """Per-operation stamps of the last k_dec_one launch made with LBIC_ONE_STAMPS=1 (lbc_one_stamps): a list of
        [first in, last inputs there, last reduced, last published] in us relative to the first operation's first entry
        (then [decode started, symbols decoded, shader clock MHz] of the rANS operation)."""
        arr = (ctypes.c_ulonglong * 52)()
        n = ctypes.c_int()
        _lib.check(_lib.lib().lbc_one_stamps(self._h, arr, 52, ctypes.byref(n)))
        v = list(arr[:n.value])
        if not v:
            return []
        t0 = min(x for x in v[0:48:4] if x) if any(v[0:48:4]) else 0
        rel = lambda x: round((x - t0) / 100.0, 2) if x and x != 2 ** 64 - 1 else None
        out = [[rel(v[4 * o + k]) for k in (0, 3, 1, 2)] for o in range(min(12, n.value // 4))]
        if n.value >= 52:
            # the rANS op: decode started (inputs in LDS), symbols decoded, and the shader clock over that span (MHz:
            # s_memtime ticks / s_memrealtime ticks x 100 MHz)
            clk = round((v[51] - v[50]) / (v[49] - v[48]) * 100.0, 1) if v[49] > v[48] and v[51] > v[50] else None
            out.append([rel(v[48]), rel(v[49]), clk])
        return out

    def one_phase_stamps(self):
        """The phases of the sampled raster step in the workgroup holding column tile 0 of each GEMM operation (the
        same launch as one_stamps): per op [in, first wave's inputs there, last wave's inputs there, last wave's A and
        weights in registers, last chain done, partials reduced, thread 0's granule store issued, published (the tile
        loop's closing barrier)] in us relative to the first operation's
        first entry, then the per-wave input times; for the rANS op [coder prologue done, symbols decoded, speculation breaks, +-1 symbols,
        searched symbols]."""
        per, words = 32, 52 + 12 * 32
        arr = (ctypes.c_ulonglong * words)()
        n = ctypes.c_int()
        _lib.check(_lib.lib().lbc_one_stamps(self._h, arr, words, ctypes.byref(n)))
        v = list(arr[:n.value])
        if len(v) < words:
            return []
        t0 = min(x for x in v[0:48:4] if x) if any(v[0:48:4]) else 0
        rel = lambda x: round((x - t0) / 100.0, 2) if x and x != 2 ** 64 - 1 else None
        out = []
        for o in range(12):
            d = v[52 + per * o: 52 + per * (o + 1)]
            if o == 4:      # the rANS op: coder prologue done, symbols done, speculation breaks, +-1, searched
                out.append([rel(d[0]), rel(d[1]), d[2], d[3], d[4]])
                continue
            rdy = [x for x in d[1:9] if x]
            mx = lambda a: max(a) if a else 0
            out.append([rel(d[0]), rel(min(rdy) if rdy else 0), rel(mx(rdy)), rel(mx(d[9:17])), rel(mx(d[17:25])),
                        rel(d[25]), rel(d[27]), rel(d[26]), [rel(x) for x in d[1:9]]])
        return out

    def rans_decode_gpu(self, streams: Sequence[bytes], indexes: torch.Tensor) -> torch.Tensor:
        """RansDecoder.decode_with_indexes (net:439) on the GPU for n streams at once: indexes [C, n, M]
        int32 (chunk c = the next M symbols of every stream, as one raster step of decompress) ->
        symbols [C, n, M] int32 on the model's device (lbc_rans_decode_gpu; the decoder's own kernel)."""
        self._check_ready()
        n = len(streams)
        idx = indexes.to(self.device, torch.int32).contiguous()
        if idx.dim() != 3 or idx.shape[1] != n or idx.shape[2] != self.arch.M:
            raise ValueError(f"indexes must be [chunks, {n}, {self.arch.M}]")
        bufs = [s if isinstance(s, bytes) else bytes(s) for s in streams]
        arr = (ctypes.c_void_p * n)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in bufs])
        lens = (ctypes.c_size_t * n)(*[len(s) for s in streams])
        sym = torch.empty_like(idx)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(_lib.lib().lbc_rans_decode_gpu(self._h, arr, lens, n, _lib.ptr(idx), idx.shape[0], _lib.ptr(sym),
                                                   ctypes.c_void_p(stream)))
        return sym

    def set_encoder_lds_floor(self, nbytes: int):
        """LBC_OPT_ENC_LDS_FLOOR: LDS reserved per encoder GEMM workgroup (> 80 KB: one per CU, leaving
        room for a decoder on another stream).  Performance only; results are unchanged."""
        _lib.check(_lib.lib().lbc_set_option(self._h, 1, int(nbytes)))

    def set_encoder_fork(self, mode: int):
        """LBC_OPT_ENC_FORK: -1 (default) the encoder graph forks its wavefront steps (context net beside the
        transform) only for passes of at most 2,048 rows per step; 0 one chain; 1 forked.  Results unchanged."""
        _lib.check(_lib.lib().lbc_set_option(self._h, 4, int(mode)))

    def validate_recu_reco(self, x: torch.Tensor):
        """The recursive reconstruction of BlockBasedImgCompLossyAgent.validate_recu_reco_fast
        (agents/blkbsdimgcomp_agent.py:491-520): raster closed loop of forward() on causal crops, i.e. the
        closed-loop encoder with forward()'s border semantics, no entropy coding.  x: [n, 3B^2, Hb, Wb].
        Returns (zhat [n, 3B^2, Hb, Wb], self_information [n, M, Hb, Wb])."""
        if x.dim() != 4 or x.shape[1] != self.arch.cx:
            raise ValueError(f"x must be [n, {self.arch.cx}, Hb, Wb]")
        n, _, Hb, Wb = x.shape
        r = self.compress_batch(x.to(self.device, torch.float32).permute(0, 2, 3, 1).contiguous(), want_bits=True,
                                frame_pad=True)
        info = r["bits"].view(n, Hb, Wb, self.arch.M).permute(0, 3, 1, 2)
        return r["zhat"].permute(0, 3, 1, 2), info

    def forward(self, zhat: torch.Tensor, x: torch.Tensor):
        """BlockBasedImgCompLossyNetv4.forward(zhat, x) (net:90-106, inherited by v9) in eval semantics:
        teacher forced on the given reconstruction, full-frame convolutions.  zhat, x: [n, 3B^2, Hb, Wb]
        (block->channel layout of arrange_block_pixels_to_channel_dim).  Returns (xhat [n, 3B^2, Hb, Wb],
        self_information [n, M, Hb, Wb] = -log2 p), like the reference; xhat is not clamped.  Needs no CDFs
        (the reference's forward() runs before update() too)."""
        if zhat.shape != x.shape or zhat.dim() != 4 or zhat.shape[1] != self.arch.cx:
            raise ValueError(f"forward expects zhat, x of shape [n, {self.arch.cx}, Hb, Wb]")
        n, _, Hb, Wb = x.shape
        xb = x.to(self.device, torch.float32).permute(0, 2, 3, 1).contiguous()
        zb = zhat.to(self.device, torch.float32).permute(0, 2, 3, 1).contiguous()
        xhat = torch.empty_like(xb)
        info = torch.empty((n, Hb, Wb, self.arch.M), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(_lib.lib().lbc_forward(self._h, _lib.ptr(xb), _lib.ptr(zb), n, Hb, Wb, _lib.ptr(xhat),
                                          _lib.ptr(info), ctypes.c_void_p(stream)))
        return xhat.permute(0, 3, 1, 2), info.permute(0, 3, 1, 2)

    __call__ = forward

    def profile_begin(self, sample_every: int):
        """Sample every n-th step's kernels with in-kernel timing stamps (lbc_profile_begin)."""
        _lib.check(_lib.lib().lbc_profile_begin(self._h, int(sample_every)))

    def profile_end(self):
        """-> {kernel family: dict(launches, total_launches, total_ms, flops, bytes, launches_chain,
        total_ms_chain)} over the sampled launches executed since profile_begin."""
        arr = (_lib.LbcKernelStat * 8)()
        n = ctypes.c_int()
        _lib.check(_lib.lib().lbc_profile_end(self._h, arr, 8, ctypes.byref(n)))
        return {arr[i].name.decode(): dict(launches=arr[i].launches, total_launches=arr[i].total_launches,
                                           total_ms=arr[i].total_ms, flops=arr[i].flops, bytes=arr[i].bytes,
                                           launches_chain=arr[i].launches_chain,
                                           total_ms_chain=arr[i].total_ms_chain, total_flops=arr[i].total_flops,
                                           total_bytes=arr[i].total_bytes)
                for i in range(n.value)}

    def last_timing(self):
        e, d = ctypes.c_double(), ctypes.c_double()
        _lib.check(_lib.lib().lbc_last_timing(self._h, ctypes.byref(e), ctypes.byref(d)))
        return e.value, d.value

    # ------------------------------------------------------------------ reference interface
    def compress(self, x, LRU, chlat):
        """net:319-361.  x: [1, 3B^2, H/B, W/B] in [-1/2, 1/2] -> (bitstream, zhat [1, 3B^2, H/B, W/B])."""
        self._check_lru(LRU)
        if chlat != self.arch.M:
            raise ValueError("chlat must equal config.M")
        if x.dim() != 4 or x.shape[0] != 1:
            raise ValueError("compress() takes one image [1, 3B^2, H/B, W/B] (the reference is batch-1)")
        xb = x.to(self.device, torch.float32).permute(0, 2, 3, 1).contiguous()
        r = self.compress_batch(xb)
        stream = self.entropy_encode(r["symbols"], r["indexes"])[0]
        return stream, r["zhat"].permute(0, 3, 1, 2).contiguous()

    def decompress(self, bitstream, LRU, xshape, chlat, devc=None):
        """net:400-452 -> zhat [1, 3B^2, H/B, W/B] on this model's device."""
        self._check_lru(LRU)
        if chlat != self.arch.M:
            raise ValueError("chlat must equal config.M")
        bt, ch, hg, wd = (int(v) for v in xshape)
        if bt != 1 or ch != self.arch.cx:
            raise ValueError("xshape must be [1, 3B^2, H/B, W/B]")
        z = self.decompress_batch([bitstream], hg, wd)
        return z.permute(0, 3, 1, 2).contiguous()


def decompress_teams(models: Sequence["BlockBasedImgCompLossyNetv9"], batches: Sequence[Sequence[bytes]], Hb: int, Wb: int,
                     wg_per_cu: int = 1, team_size: int = 0):
    """Decode len(batches) <= 16 batches of reference-format bitstreams in ONE persistent launch (lbc_decode_team: one
    team of workgroups per batch on one XCD; more than 8 batches: two teams per XCD, each half its CUs):
    batch t by models[t] (distinct handles of one geometry, e.g. siblings), each batch the same number of images of
    Hb x Wb blocks.  Returns [zhat_t [n, Hb, Wb, 3B^2]], bit-identical to models[t].decompress_batch(batches[t]).
    wg_per_cu (LBC_OPT_TEAM_WG_PER_CU): 1 leaves room for an encoder running beside the launch; 2 doubles each
    team's workgroups (every register of the GPU) for a decode with the GPU otherwise idle.  team_size
    (LBC_OPT_TEAM_SIZE): workgroups per team, 0 = one per CU of an XCD; fewer: small teams."""
    T = len(batches)
    if T < 1 or T > 16 or len(models) < T:
        raise ValueError("1 to 16 batches, one model handle each")
    n = len(batches[0])
    if any(len(b) != n for b in batches):
        raise ValueError("every batch needs the same number of images")
    for m in models[:T]:
        m._check_ready()
    bufs = [s if isinstance(s, bytes) else bytes(s) for b in batches for s in b]
    arr = (ctypes.c_void_p * len(bufs))(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in bufs])
    lens = (ctypes.c_size_t * len(bufs))(*[len(b) for b in bufs])
    dev = models[0].device
    zh = [torch.empty((n, Hb, Wb, models[0].arch.cx), dtype=torch.float32, device=dev) for _ in range(T)]
    hs = (ctypes.c_void_p * T)(*[m._h for m in models[:T]])
    zp = (ctypes.c_void_p * T)(*[_lib.ptr(z) for z in zh])
    stream = torch.cuda.current_stream(dev).cuda_stream
    _lib.check(_lib.lib().lbc_set_option(models[0]._h, 2, int(wg_per_cu)))
    _lib.check(_lib.lib().lbc_set_option(models[0]._h, 3, int(team_size)))
    _lib.check(_lib.lib().lbc_decode_team(hs, T, arr, lens, n, Hb, Wb, zp, ctypes.c_void_p(stream)))
    return zh
