"""Layer geometry of ``BlockBasedImgCompLossyNetv9`` and the reference state-dict names.

Mirrors the constructor at graphs/models/BlockBasedImgCompLossy_net.py:259-317 (v9 overrides the v4
modules created by ``super().__init__`` at :21-66, keeping v4's registration order, hence the
state-dict key order below).  Only geometry lives here; no arithmetic.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

# Causal taps of a 3x3 'A' mask, graphs/layers/masked_conv2d.py:9-17: the row above (3 taps) and the
# left neighbour.  A 3x3 'B' mask adds the centre.  (dy, dx) relative to the output position.
TAPS_A3 = ((-1, -1), (-1, 0), (-1, 1), (0, -1))
TAPS_B3 = TAPS_A3 + ((0, 0),)


@dataclass(frozen=True)
class Arch:
    B: int            # block size (configs/*.json "block_size")
    KS: Tuple[int, int, int, int]
    N: int
    M: int

    @property
    def cx(self) -> int:          # channels of one block in the block->channel layout (3*B^2)
        return 3 * self.B * self.B

    @property
    def n7(self) -> int:
        return self.N // 8 * 7

    @property
    def n6(self) -> int:
        return self.N // 8 * 6

    @property
    def c_ctx(self) -> Tuple[int, int, int, int]:   # get_meanscale widths, net:296-302
        return (self.N // 8 * 12, self.N // 8 * 10, self.N // 8 * 8, self.M * 2)

    @property
    def lru(self) -> int:
        """L = R = U for compress/decompress, agents/blkbsdimgcomp_agent.py:481-489."""
        return sum(k // 2 for k in self.KS)

    @property
    def ctx_positions(self):
        """Layer-0 output positions the context net's second layer consumes (window semantics)."""
        return TAPS_B3 if self.KS[1] == 3 else ((0, 0),)

    def conv_specs(self) -> List[Tuple[str, str, int, int, int]]:
        """(module, mask_type, cin, cout, k) for every MaskedConv2d in state-dict order."""
        cx, N, M = self.cx, self.N, self.M
        K1 = self.KS[0]
        c1, c2, c3, c4 = self.c_ctx
        return [
            ("prtr_forward1", "B", cx, N, 1),
            ("prtr_forward2", "A", cx, N, K1),
            ("prtr_forward3.1", "B", N, self.n7, 1),
            ("prtr_forward3.3", "B", self.n7, self.n6, 1),
            ("prtr_forward3.5", "B", self.n6, M, 1),
            ("prtr_inverse1", "B", M, N, 1),
            ("prtr_inverse2", "A", cx, N, K1),
            ("prtr_inverse3.1", "B", N, self.n7, 1),
            ("prtr_inverse3.3", "B", self.n7, self.n6, 1),
            ("prtr_inverse3.5", "B", self.n6, cx, 1),
            ("get_meanscale.0", "A", cx, c1, K1),
            ("get_meanscale.2", "B", c1, c2, self.KS[1]),
            ("get_meanscale.4", "B", c2, c3, 1),
            ("get_meanscale.6", "B", c3, c4, 1),
        ]

    def gdn_specs(self) -> List[Tuple[str, int, bool]]:
        """(module, channels, inverse) for every GDN in state-dict order."""
        N = self.N
        return [
            ("prtr_forward3.0", N, False), ("prtr_forward3.2", self.n7, False), ("prtr_forward3.4", self.n6, False),
            ("prtr_inverse3.0", N, True), ("prtr_inverse3.2", self.n7, True), ("prtr_inverse3.4", self.n6, True),
        ]

    def param_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """Trainable parameters (weight/bias/beta/gamma) in the reference's state-dict order."""
        convs = {c[0]: c for c in self.conv_specs()}
        gdns = {g[0]: g for g in self.gdn_specs()}
        order = ["prtr_forward1", "prtr_forward2", "prtr_forward3.0", "prtr_forward3.1", "prtr_forward3.2",
                 "prtr_forward3.3", "prtr_forward3.4", "prtr_forward3.5", "prtr_inverse1", "prtr_inverse2",
                 "prtr_inverse3.0", "prtr_inverse3.1", "prtr_inverse3.2", "prtr_inverse3.3", "prtr_inverse3.4",
                 "prtr_inverse3.5", "get_meanscale.0", "get_meanscale.2", "get_meanscale.4", "get_meanscale.6"]
        out = []
        for name in order:
            if name in convs:
                _, _, cin, cout, k = convs[name]
                out.append((name + ".weight", (cout, cin, k, k)))
                out.append((name + ".bias", (cout,)))
            else:
                _, c, _ = gdns[name]
                out.append((name + ".beta", (c,)))
                out.append((name + ".gamma", (c, c)))
        return out

    def live_macs_per_block(self) -> Tuple[int, int]:
        """Live (unmasked) MACs per block: (encoder incl. context + decoder transform, decoder = context +
        decoder transform).  Used for the algorithmic FLOP count."""
        ntap = 4 if self.KS[0] == 3 else 0
        cx, N, M = self.cx, self.N, self.M
        c1, c2, c3, c4 = self.c_ctx
        P = len(self.ctx_positions)
        ctx = P * ntap * cx * c1 + (5 if self.KS[1] == 3 else 1) * c1 * c2 + c2 * c3 + c3 * c4
        gdn = N * N + self.n7 * self.n7 + self.n6 * self.n6
        fwd = (ntap * cx + cx) * N + N * self.n7 + self.n7 * self.n6 + self.n6 * M + gdn
        inv = (ntap * cx + M) * N + N * self.n7 + self.n7 * self.n6 + self.n6 * cx + gdn
        return fwd + ctx + inv, ctx + inv


def arch_from_config(config) -> Arch:
    return Arch(int(config.block_size), tuple(int(k) for k in config.KS), int(config.N), int(config.M))
