"""ORACLE -- test infrastructure, never the product.

CPU restatement (numpy fp32 + plain C for the entropy coder) of the reference's block-level closed-loop
codec, ``BlockBasedImgCompLossyNetv9.compress`` / ``decompress``
(graphs/models/BlockBasedImgCompLossy_net.py:319-452 in /root/reference).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module, and only as
the checker / CPU baseline.

Pinned against the golden vectors in tests/golden/ that were produced by the reference's own Python
(tests/golden/gen_golden.py): per-stage activations (tolerance 1e-5 rel), closed-loop symbols and scale
indexes (bit-exact on tie-screened fixtures), reconstructions (1e-5), scale table and pmfs.  The
quantized CDFs and rANS bytes follow CompressAI's published algorithm (oracle/rans_oracle.c): parity
unpinned, no reference fixture holds them.

Conventions: one image at a time, block-major layout [Hb, Wb, C] with C = 3*B^2 (channel index
(py*B + px)*3 + colour, agents/blkbsdimgcomp_agent.py:853-860).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
F32 = np.float32

TAPS_A3 = ((-1, -1), (-1, 0), (-1, 1), (0, -1))       # masked_conv2d.py:9-17, 'A' 3x3
TAPS_B3 = TAPS_A3 + ((0, 0),)

_LIB = None


def _lib():
    """Build (if needed) and load oracle/build/liboracle.so."""
    global _LIB
    if _LIB is None:
        so = os.path.join(HERE, "build", "liboracle.so")
        src = os.path.join(HERE, "rans_oracle.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", HERE])
        lib = ctypes.CDLL(so)
        P = ctypes.c_void_p
        lib.oracle_pmf_to_quantized_cdf.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
        lib.oracle_rans_encode.argtypes = [P, P, ctypes.c_long, P, ctypes.c_int, P, P, ctypes.c_int, P,
                                           ctypes.c_long]
        lib.oracle_rans_encode.restype = ctypes.c_long
        lib.oracle_dec_new.argtypes = [P, ctypes.c_long]
        lib.oracle_dec_new.restype = P
        lib.oracle_dec_free.argtypes = [P]
        lib.oracle_dec_decode.argtypes = [P, P, ctypes.c_long, P, ctypes.c_int, P, P, ctypes.c_int, P]
        _LIB = lib
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---------------------------------------------------------------------------------- entropy model
def scale_table():
    """get_scale_table(), net:13-18: exp(linspace(ln .11, ln 256, 64)) in float32, restating torch's CPU
    linspace bit for bit (first half: vectorised base + step*j per 8-lane chunk; second half:
    end - step*(n-1-i) fused into one rounding) and a correctly rounded exp."""
    n, vec = 64, 8
    start, end = F32(math.log(0.11)), F32(math.log(256))
    step = F32((end - start) / F32(n - 1))
    lin = np.zeros(n, F32)
    for i in range(n):
        if i < n // 2:
            base = F32(start + F32(step * F32(i - i % vec)))
            lin[i] = F32(base + F32(step * F32(i % vec)))
        else:   # fma: the product of a 24-bit and a 6-bit value and this sum are exact in float64
            lin[i] = F32(np.float64(end) - np.float64(step) * (n - 1 - i))
    return np.exp(lin.astype(np.float64)).astype(F32)


def _erfc32(x):
    from scipy.special import erfc
    return erfc(x.astype(np.float64)).astype(F32)


def std_cumulative(x):
    """_standardized_cumulative, entropy_layers_cai.py:569-573: 0.5 * erfc(-(2**-0.5) * x)."""
    return (F32(0.5) * _erfc32(F32(-(2 ** -0.5)) * x)).astype(F32)


def gaussian_pmfs(table, tail_mass=1e-9):
    """GaussianConditional.update, entropy_layers_cai.py:590-613, up to the pmf_to_quantized_cdf call:
    returns (prob list [pmf[:len] + tail], offset, cdf_length)."""
    from scipy.stats import norm
    multiplier = -norm.ppf(tail_mass / 2)
    center = np.ceil(table.astype(F32) * F32(multiplier)).astype(np.int32)
    length = 2 * center + 1
    maxlen = int(length.max())
    samples = np.abs(np.arange(maxlen, dtype=np.int32)[None, :] - center[:, None]).astype(F32)
    sc = table[:, None].astype(F32)
    upper = std_cumulative((F32(0.5) - samples) / sc)
    lower = std_cumulative((F32(-0.5) - samples) / sc)
    pmf = (upper - lower).astype(F32)
    tail = (F32(2) * lower[:, :1]).astype(F32)
    probs = [np.concatenate([pmf[i, :length[i]], tail[i]]).astype(F32) for i in range(len(table))]
    return probs, (-center).astype(np.int32), (length + 2).astype(np.int32)


def pmf_to_quantized_cdf(prob, precision=16):
    prob = np.ascontiguousarray(prob, F32)
    out = np.zeros(len(prob) + 1, np.uint32)
    rc = _lib().oracle_pmf_to_quantized_cdf(_p(prob), len(prob), precision, _p(out))
    if rc != 0:
        raise ValueError(f"pmf_to_quantized_cdf failed ({rc})")
    return out.astype(np.int32)


class GaussianTables:
    """scale table + quantized CDF rows, offsets, lengths (the buffers update() fills)."""

    def __init__(self, probs=None):
        self.table = scale_table()
        p, self.offset, self.cdf_length = gaussian_pmfs(self.table)
        probs = p if probs is None else probs
        maxlen = int(self.cdf_length.max())
        self.cdf = np.zeros((len(probs), maxlen), np.int32)
        for i, pr in enumerate(probs):
            c = pmf_to_quantized_cdf(pr)
            self.cdf[i, :len(c)] = c

    def encode(self, symbols, indexes):
        s = np.ascontiguousarray(symbols, np.int32)
        ix = np.ascontiguousarray(indexes, np.int32)
        cap = 64 + 8 * len(s)
        buf = np.zeros(cap, np.uint8)
        n = _lib().oracle_rans_encode(_p(s), _p(ix), len(s), _p(self.cdf), self.cdf.shape[1], _p(self.cdf_length),
                                      _p(self.offset), len(self.offset), _p(buf), cap)
        if n < 0:
            raise RuntimeError(f"rans encode failed {n}")
        return bytes(buf[:n])

    def decoder(self, data):
        return _Decoder(self, data)


class _Decoder:
    def __init__(self, tabs, data):
        self.t = tabs
        self.buf = np.frombuffer(bytes(data) + b"\0" * 8, np.uint8).copy()
        self.h = _lib().oracle_dec_new(_p(self.buf), len(data))

    def decode_stream(self, indexes):
        ix = np.ascontiguousarray(indexes, np.int32)
        out = np.zeros(len(ix), np.int32)
        rc = _lib().oracle_dec_decode(self.h, _p(ix), len(ix), _p(self.t.cdf), self.t.cdf.shape[1],
                                      _p(self.t.cdf_length), _p(self.t.offset), len(self.t.offset), _p(out))
        if rc != 0:
            raise RuntimeError("rans decode failed")
        return out

    def __del__(self):
        if getattr(self, "h", None):
            _lib().oracle_dec_free(self.h)
            self.h = None


def build_indexes(scales, table):
    """entropy_layers_cai.py:649-654."""
    s = np.maximum(scales.astype(F32), F32(0.11))
    idx = np.full(s.shape, len(table) - 1, np.int32)
    for t in table[:-1]:
        idx -= (s <= t).astype(np.int32)
    return idx


def likelihood_bits(yq, scales, means):
    """_likelihood + LowerBound(1e-9) + (-log2), entropy_layers_cai.py:615-647, net:103."""
    v = np.abs((yq - means).astype(F32))
    s = np.maximum(scales.astype(F32), F32(0.11))
    upper = std_cumulative((F32(0.5) - v) / s)
    lower = std_cumulative((F32(-0.5) - v) / s)
    lik = np.maximum((upper - lower).astype(F32), F32(1e-9))
    return (-np.log2(lik)).astype(F32)


# ---------------------------------------------------------------------------------- transforms
def _leaky(x):
    return np.where(x > 0, x, x * F32(0.01)).astype(F32)


class OracleNet:
    """Weights prepared exactly as the reference applies them: weight*mask (masked_conv2d.py:19-21,
    net:380-397) and the GDN non-negative reparametrisation (gdn_compressai.py:66-68,
    utils/parametrizers.py:45-47)."""

    def __init__(self, arch, sd):
        self.a = arch
        self.sd = sd
        B = arch.B
        self.cx = 3 * B * B
        self.conv = {}
        for name, mtype, cin, cout, k in arch.conv_specs():
            w = sd[name + ".weight"].astype(F32)
            b = sd[name + ".bias"].astype(F32)
            if k == 1:
                self.conv[name] = ([w[:, :, 0, 0]], b)                       # [cout, cin]
            else:
                taps = TAPS_A3 if mtype == "A" else TAPS_B3
                self.conv[name] = ([np.ascontiguousarray(w[:, :, 1 + dy, 1 + dx]) for dy, dx in taps], b)
        self.gdn = {}
        ped = F32(2.0 ** -18) ** 2
        for name, c, inv in arch.gdn_specs():
            bb = F32((1e-6 + float(ped)) ** 0.5)
            gb = F32((0.0 + float(ped)) ** 0.5)
            beta = (np.maximum(sd[name + ".beta"].astype(F32), bb) ** 2 - ped).astype(F32)
            gamma = (np.maximum(sd[name + ".gamma"].astype(F32), gb) ** 2 - ped).astype(F32)
            self.gdn[name] = (beta, gamma, inv)

    def _lin(self, name, vecs):
        ws, b = self.conv[name]
        acc = b.copy()
        for w, v in zip(ws, vecs):
            acc = acc + w @ v
        return acc.astype(F32)

    def _gdn(self, name, x):
        beta, gamma, inv = self.gdn[name]
        norm = (gamma @ (x * x) + beta).astype(F32)
        r = np.sqrt(norm) if inv else F32(1.0) / np.sqrt(norm)
        return (x * r.astype(F32)).astype(F32)

    @staticmethod
    def _taps(win, c, taps):
        """win: [2L+1, 2L+1, C] window, c: (row, col) of the output position inside it."""
        return [win[c[0] + dy, c[1] + dx] for dy, dx in taps]

    def ctx(self, win, inside=None):
        """get_meanscale_fast (net:389-398) on a (2L+1)^2 zero-padded window (valid convs).  inside: for
        KS[1] = 3, a predicate on the layer-1 tap offsets (dy, dx); taps outside the frame contribute a zero
        layer-0 vector (forward()'s 'same' zero padding, used by validate_recu_reco_fast), default: the
        layer-0 map is evaluated on the zero-padded window (compress())."""
        L = win.shape[0] // 2
        a = self.a
        if a.KS[1] == 3:
            l0 = [_leaky(self._lin("get_meanscale.0", self._taps(win, (L + dy, L + dx), TAPS_A3)))
                  if inside is None or inside(dy, dx) else np.zeros_like(self.conv["get_meanscale.0"][1])
                  for dy, dx in TAPS_B3]
            l1 = _leaky(self._lin("get_meanscale.2", l0))
        else:
            l0 = _leaky(self._lin("get_meanscale.0", self._taps(win, (L, L), TAPS_A3)))
            l1 = _leaky(self._lin("get_meanscale.2", [l0]))
        l2 = _leaky(self._lin("get_meanscale.4", [l1]))
        return self._lin("get_meanscale.6", [l2])

    def fwd(self, win, x):
        """forward_prtr_fast (net:379-382): 1x1 on x + masked 3x3 on the centre of the window."""
        L = win.shape[0] // 2
        z = self._taps(win, (L, L), TAPS_A3)
        h = (self._lin("prtr_forward1", [x]) + self._lin("prtr_forward2", z)).astype(F32)
        h = self._gdn("prtr_forward3.0", h)
        h = self._gdn("prtr_forward3.2", self._lin("prtr_forward3.1", [h]))
        h = self._gdn("prtr_forward3.4", self._lin("prtr_forward3.3", [h]))
        return self._lin("prtr_forward3.5", [h])

    def inv(self, win, yq):
        """inverse_prtr_fast (net:384-387)."""
        L = win.shape[0] // 2
        z = self._taps(win, (L, L), TAPS_A3)
        h = (self._lin("prtr_inverse1", [yq]) + self._lin("prtr_inverse2", z)).astype(F32)
        h = self._gdn("prtr_inverse3.0", h)
        h = self._gdn("prtr_inverse3.2", self._lin("prtr_inverse3.1", [h]))
        h = self._gdn("prtr_inverse3.4", self._lin("prtr_inverse3.3", [h]))
        return self._lin("prtr_inverse3.5", [h])


    def forward_frame(self, zhat, x):
        """forward(zhat, x) (net:90-106, inherited by v9; eval mode): teacher forced on a given zhat with the
        full-frame 'same' convolutions of the nn.Sequential layers.  Differs from the closed loop only for
        KS[1] = 3, where the 3x3 'B' layer of get_meanscale zero-pads the layer-0 MAP at the frame border
        (the closed loop evaluates layer 0 on the zero-padded zhat there).  zhat, x: [Hb, Wb, C].
        Returns xhat [Hb, Wb, C] (not clamped) and self-information -log2 p [Hb, Wb, M]."""
        a = self.a
        Hb, Wb, C = zhat.shape
        zp = np.zeros((Hb + 2, Wb + 2, C), F32)
        zp[1:-1, 1:-1] = zhat
        l0 = np.zeros((Hb, Wb, self.conv["get_meanscale.0"][1].shape[0]), F32)
        for v in range(Hb):
            for h in range(Wb):
                l0[v, h] = _leaky(self._lin("get_meanscale.0", self._taps(zp, (v + 1, h + 1), TAPS_A3)))
        l0p = np.zeros((Hb + 2, Wb + 2, l0.shape[2]), F32)
        l0p[1:-1, 1:-1] = l0
        xhat = np.zeros_like(zhat)
        info = np.zeros((Hb, Wb, a.M), F32)
        for v in range(Hb):
            for h in range(Wb):
                if a.KS[1] == 3:
                    l1 = _leaky(self._lin("get_meanscale.2", self._taps(l0p, (v + 1, h + 1), TAPS_B3)))
                else:
                    l1 = _leaky(self._lin("get_meanscale.2", [l0[v, h]]))
                l2 = _leaky(self._lin("get_meanscale.4", [l1]))
                ksi = self._lin("get_meanscale.6", [l2])
                scales, means = ksi[:a.M], ksi[a.M:]
                win = zp[v:v + 3, h:h + 3]
                y = self.fwd(win, x[v, h])
                yq = (np.rint((y - means).astype(F32)) + means).astype(F32)   # quantize(..., "dequantize")
                info[v, h] = likelihood_bits(yq, scales, means)
                xhat[v, h] = self.inv(win, yq)
        return xhat, info


class OracleCodec:
    """compress()/decompress() of the reference, one image, raster closed loop."""

    def __init__(self, arch, sd, tables=None):
        self.a = arch
        self.net = OracleNet(arch, sd)
        self.tabs = tables if tables is not None else GaussianTables()

    def _window(self, zp, v, h):
        L = self.a.lru
        return zp[v:v + 2 * L + 1, h:h + 2 * L + 1]

    def code_block(self, zp, v, h, x, frame=None):
        """compress_blk (net:363-377) + clamp (net:357): returns sym, idx, yq, bits, xhat.  frame = (Hb, Wb):
        forward()'s border semantics for the context net (validate_recu_reco_fast)."""
        M = self.a.M
        win = self._window(zp, v, h)
        inside = None
        if frame is not None:
            inside = lambda dy, dx: 0 <= v + dy < frame[0] and 0 <= h + dx < frame[1]
        ksi = self.net.ctx(win, inside)
        scales, means = ksi[:M], ksi[M:]
        idx = build_indexes(scales, self.tabs.table)
        y = self.net.fwd(win, x)
        sym = np.rint((y - means).astype(F32)).astype(np.int32)
        yq = (sym.astype(F32) + means).astype(F32)
        bits = likelihood_bits(yq, scales, means)
        xhat = np.clip(self.net.inv(win, yq), F32(-0.5), F32(0.5)).astype(F32)
        return sym, idx, yq, bits, xhat

    def validate_recu(self, x):
        """validate_recu_reco_fast (agent:491-520): the raster closed loop of forward() on causal crops, which
        is compress()'s loop with forward()'s zero padding of the context layer-0 map at the frame border.
        x: [Hb, Wb, C].  Returns (zhat [Hb, Wb, C], self-information [Hb, Wb, M])."""
        Hb, Wb, C = x.shape
        L = self.a.lru
        zp = np.zeros((Hb + 2 * L, Wb + 2 * L, C), F32)
        info = np.zeros((Hb, Wb, self.a.M), F32)
        for v in range(Hb):
            for h in range(Wb):
                _, _, _, bits, xhat = self.code_block(zp, v, h, x[v, h], frame=(Hb, Wb))
                zp[v + L, h + L] = xhat
                info[v, h] = bits
        return zp[L:L + Hb, L:L + Wb].copy(), info

    def compress(self, x, rows=None, with_bytes=True):
        """x: [Hb, Wb, C] fp32.  Returns dict(bytes, zhat, symbols [Hb*Wb*M], indexes, bits).
        ``rows`` limits the loop to the first rows (CPU-baseline sample)."""
        Hb, Wb, C = x.shape
        L = self.a.lru
        rows = Hb if rows is None else rows
        zp = np.zeros((Hb + 2 * L, Wb + 2 * L, C), F32)
        syms, idxs, bits = [], [], []
        for v in range(rows):
            for h in range(Wb):
                s, i, _, b, xh = self.code_block(zp, v, h, x[v, h])
                syms.append(s), idxs.append(i), bits.append(b)
                zp[v + L, h + L] = xh
        sy, ix = np.concatenate(syms), np.concatenate(idxs)
        out = dict(zhat=zp[L:L + Hb, L:L + Wb].copy(), symbols=sy, indexes=ix, bits=np.concatenate(bits))
        if with_bytes:
            out["bytes"] = self.tabs.encode(sy, ix)
        return out

    def decompress(self, data, Hb, Wb, rows=None):
        """decompress() (net:400-452): strictly raster serial, rANS decode per block."""
        a = self.a
        L, M, C = a.lru, a.M, a.cx
        rows = Hb if rows is None else rows
        zp = np.zeros((Hb + 2 * L, Wb + 2 * L, C), F32)
        dec = self.tabs.decoder(data)
        for v in range(rows):
            for h in range(Wb):
                win = self._window(zp, v, h)
                ksi = self.net.ctx(win)
                scales, means = ksi[:M], ksi[M:]
                idx = build_indexes(scales, self.tabs.table)
                sym = dec.decode_stream(idx)
                yq = (sym.astype(F32) + means).astype(F32)
                zp[v + L, h + L] = np.clip(self.net.inv(win, yq), F32(-0.5), F32(0.5))
        return zp[L:L + Hb, L:L + Wb].copy()


# ---------------------------------------------------------------------------------- layout
def image_to_blocks(img_chw, B):
    """arrange_block_pixels_to_channel_dim (agents/blkbsdimgcomp_agent.py:853-860) for one image,
    returning the block-major [Hb, Wb, 3B^2] layout."""
    C, H, W = img_chw.shape
    x = img_chw.reshape(C, H // B, B, W // B, B)              # c, vb, py, hb, px
    return np.ascontiguousarray(x.transpose(1, 3, 2, 4, 0).reshape(H // B, W // B, B * B * C))


def blocks_to_image(xb, B):
    Hb, Wb, CC = xb.shape
    C = CC // (B * B)
    x = xb.reshape(Hb, Wb, B, B, C).transpose(4, 0, 2, 1, 3)
    return np.ascontiguousarray(x.reshape(C, Hb * B, Wb * B))
