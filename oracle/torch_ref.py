"""ORACLE -- test infrastructure and CPU baseline, never the product.

Torch-CPU restatement of the reference's closed-loop codec as the reference executes it: per block,
small valid ``conv2d`` calls on the zero-padded reconstruction window (the MaskedConv2d layers with
their masks applied, masked_conv2d.py:9-21), GDN / IGDN as a 1x1 conv over x^2 with the
non-negative reparametrisation (gdn_compressai.py:65-80, utils/parametrizers.py:42-47), the context
net on the (2L+1)^2 window (get_meanscale_fast, graphs/models/BlockBasedImgCompLossy_net.py:389-398),
quantize / build_indexes (entropy_layers_cai.py:126-168, 649-654) and the raster loops of
``compress`` (net:319-361) and ``decompress`` (net:400-452).  Entropy coding uses the plain-C coder of
oracle/rans_oracle.c (CompressAI's format).

Used by bench.py's ``cpu_baseline`` leg: the reference's Python cannot travel to the GPU box, so this
restatement (same algorithm, same torch CPU kernels, parity-checked against the reference's golden
vectors in tests/test_oracle_golden.py) is timed there on the host cores, at 1 thread (the setting
eval_model uses, agents/blkbsdimgcomp_agent.py:565-566) and at all the threads the box grants.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import oracle as O

TAPS_A3 = O.TAPS_A3
TAPS_B3 = O.TAPS_B3


def _mask(k, mtype):
    m = torch.zeros(k, k)
    if k == 1:
        m[0, 0] = 1.0
        return m
    for dy, dx in (TAPS_A3 if mtype == "A" else TAPS_B3):
        m[1 + dy, 1 + dx] = 1.0
    return m


class TorchRef:
    """One model on the CPU.  sd: the reference state-dict names -> numpy arrays."""

    def __init__(self, arch, sd, tables=None):
        self.a = arch
        self.w = {}
        for name, mtype, cin, cout, k in arch.conv_specs():
            w = torch.from_numpy(np.asarray(sd[name + ".weight"], np.float32)) * _mask(k, mtype)
            self.w[name] = (w.contiguous(), torch.from_numpy(np.asarray(sd[name + ".bias"], np.float32)))
        ped = float(2.0 ** -18) ** 2
        self.gdn = {}
        for name, c, inv in arch.gdn_specs():
            bb = torch.tensor((1e-6 + ped) ** 0.5, dtype=torch.float32)
            gb = torch.tensor((0.0 + ped) ** 0.5, dtype=torch.float32)
            beta = torch.maximum(torch.from_numpy(np.asarray(sd[name + ".beta"], np.float32)), bb) ** 2 - ped
            gamma = torch.maximum(torch.from_numpy(np.asarray(sd[name + ".gamma"], np.float32)), gb) ** 2 - ped
            self.gdn[name] = (gamma[:, :, None, None].contiguous(), beta.contiguous(), inv)
        self.tabs = tables if tables is not None else O.GaussianTables()
        self.table = torch.from_numpy(self.tabs.table)

    # ------------------------------------------------------------------ layers
    def _conv(self, name, x):
        w, b = self.w[name]
        return F.conv2d(x, w, b)

    def _gdn(self, name, x):
        gamma, beta, inv = self.gdn[name]
        norm = F.conv2d(x * x, gamma, beta)
        return x * (torch.sqrt(norm) if inv else torch.rsqrt(norm))

    def ctx(self, win):
        """get_meanscale_fast on the (2L+1)^2 window [1, C, 2L+1, 2L+1] -> [1, 2M, 1, 1]."""
        h = F.leaky_relu(self._conv("get_meanscale.0", win), 0.01)
        h = F.leaky_relu(self._conv("get_meanscale.2", h), 0.01)
        h = F.leaky_relu(self._conv("get_meanscale.4", h), 0.01)
        return self._conv("get_meanscale.6", h)

    def fwd(self, x, z3):
        """forward_prtr_fast: x [1, C, 1, 1], z3 the centre 3x3 of the window."""
        h = self._conv("prtr_forward1", x) + self._conv("prtr_forward2", z3)
        h = self._gdn("prtr_forward3.0", h)
        h = self._gdn("prtr_forward3.2", self._conv("prtr_forward3.1", h))
        h = self._gdn("prtr_forward3.4", self._conv("prtr_forward3.3", h))
        return self._conv("prtr_forward3.5", h)

    def inv(self, yq, z3):
        """inverse_prtr_fast."""
        h = self._conv("prtr_inverse1", yq) + self._conv("prtr_inverse2", z3)
        h = self._gdn("prtr_inverse3.0", h)
        h = self._gdn("prtr_inverse3.2", self._conv("prtr_inverse3.1", h))
        h = self._gdn("prtr_inverse3.4", self._conv("prtr_inverse3.3", h))
        return self._conv("prtr_inverse3.5", h)

    def _indexes(self, scales):
        s = torch.clamp(scales, min=0.11)
        return (len(self.table) - 1 - (s[..., None] <= self.table[:-1]).sum(-1)).to(torch.int32)

    # ------------------------------------------------------------------ closed loops
    @torch.no_grad()
    def compress(self, xb, rows=None):
        """xb: [Hb, Wb, C] numpy (block-major) -> dict(bytes, symbols, indexes, zhat [Hb, Wb, C])."""
        Hb, Wb, C = xb.shape
        L, M = self.a.lru, self.a.M
        rows = Hb if rows is None else rows
        x = torch.from_numpy(np.ascontiguousarray(xb)).permute(2, 0, 1)[None]        # [1, C, Hb, Wb]
        zp = torch.zeros(1, C, Hb + 2 * L, Wb + 2 * L)
        syms, idxs = [], []
        for v in range(rows):
            for h in range(Wb):
                win = zp[:, :, v:v + 2 * L + 1, h:h + 2 * L + 1]
                ksi = self.ctx(win)
                scales, means = ksi[:, :M], ksi[:, M:]
                z3 = win[:, :, L - 1:L + 2, L - 1:L + 2]
                y = self.fwd(x[:, :, v:v + 1, h:h + 1], z3)
                sym = torch.round(y - means)
                yq = sym + means
                zp[:, :, v + L:v + L + 1, h + L:h + L + 1] = torch.clamp(self.inv(yq, z3), -0.5, 0.5)
                syms.append(sym.reshape(-1).to(torch.int32))
                idxs.append(self._indexes(scales.reshape(-1)))
        sy, ix = torch.cat(syms).numpy(), torch.cat(idxs).numpy()
        return dict(bytes=self.tabs.encode(sy, ix), symbols=sy, indexes=ix,
                    zhat=zp[0, :, L:L + Hb, L:L + Wb].permute(1, 2, 0).numpy().copy())

    @torch.no_grad()
    def decompress(self, data, Hb, Wb, rows=None):
        L, M, C = self.a.lru, self.a.M, self.a.cx
        rows = Hb if rows is None else rows
        zp = torch.zeros(1, C, Hb + 2 * L, Wb + 2 * L)
        dec = self.tabs.decoder(data)
        for v in range(rows):
            for h in range(Wb):
                win = zp[:, :, v:v + 2 * L + 1, h:h + 2 * L + 1]
                ksi = self.ctx(win)
                scales, means = ksi[:, :M], ksi[:, M:]
                sym = dec.decode_stream(self._indexes(scales.reshape(-1)).numpy())
                yq = torch.from_numpy(sym.astype(np.float32)).reshape(1, M, 1, 1) + means
                z3 = win[:, :, L - 1:L + 2, L - 1:L + 2]
                zp[:, :, v + L:v + L + 1, h + L:h + L + 1] = torch.clamp(self.inv(yq, z3), -0.5, 0.5)
        return zp[0, :, L:L + Hb, L:L + Wb].permute(1, 2, 0).numpy().copy()
