"""Calibrate lbic.weights.MID_POINTS (rate="mid": the high-rate configs' published operating points, ~1.6 bpp) with
the CPU oracle's closed loop (oracle/torch_ref.py: compress() of a seeded uint8 noise frame, C rANS bytes).

For each architecture: the latent gain g is searched (bisection on log g) so that the frame codes at the target bpp,
with the scale level s = r g, r the measured spread of the quantised residual at g = 1 (scales matched to the
residual, as a trained model's).  Prints the MID_POINTS entries to paste into lbic/weights.py.  Test infrastructure (imports the
oracle), not product code.

    python tests/golden/tune_mid_rate.py
"""
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "learned-block-based-image-compression_amd")]

from lbic.arch import Arch  # noqa: E402
from lbic.weights import synth_state_dict  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.torch_ref import TorchRef  # noqa: E402

TARGETS = {   # arch -> published bpp
    Arch(8, (3, 3, 1, 1), 1152, 128): 1.63,
    Arch(4, (3, 3, 1, 1), 512, 96): 1.58,
}
SIZE = 64
LOW_TARGETS = {   # rate="low": arch -> published bpp (B16_lowrate: 0.1200); frame size
    Arch(16, (3, 1, 1, 1), 1280, 192): (0.120, 128),
}


def code(arch, g, s, xb, rate="mid"):
    ref = TorchRef(arch, synth_state_dict(arch, 1337, rate=rate, mid=(g, s)))
    out = ref.compress(xb)
    bpp = len(out["bytes"]) * 8.0 / (xb.shape[0] * xb.shape[1] * arch.B * arch.B)
    return bpp, out


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for arch, (target, size) in LOW_TARGETS.items():
        img = np.random.default_rng(0).integers(0, 256, (3, size, size), dtype=np.uint8).astype(np.float32) / 255 - 0.5
        xb = O.image_to_blocks(img, arch.B)
        lo, hi = math.log(0.05), math.log(20.0)
        for it in range(12):
            g = math.exp(0.5 * (lo + hi))
            bpp, _ = code(arch, g, 0.0, xb, rate="low")
            print(f"{arch} low: g={g:.4f} -> {bpp:.4f} bpp (target {target})", flush=True)
            if bpp > target:
                hi = math.log(g)
            else:
                lo = math.log(g)
        print(f"LOW_POINTS[({arch.B}, {arch.N}, {arch.M})] = {g:.4f}  # {bpp:.4f} bpp on {size}x{size} noise")
    if "low" in sys.argv[1:]:
        return
    for arch, target in TARGETS.items():
        img = np.random.default_rng(0).integers(0, 256, (3, SIZE, SIZE), dtype=np.uint8).astype(np.float32) / 255 - 0.5
        xb = O.image_to_blocks(img, arch.B)
        # matched scales: the residual's spread is proportional to the gain; measure it once at g = 1 (rms of the
        # quantised residual y - mean) and keep s = r g during the search
        _, out = code(arch, 1.0, 0.3, xb)
        r = float(np.sqrt(np.mean(out["symbols"].astype(np.float64) ** 2)))
        lo, hi = math.log(0.05), math.log(20.0)
        for it in range(12):
            g = math.exp(0.5 * (lo + hi))
            s = max(r * g, 0.11)
            bpp, out = code(arch, g, s, xb)
            print(f"{arch}: g={g:.4f} s={s:.4f} -> {bpp:.4f} bpp (target {target})", flush=True)
            if bpp > target:
                hi = math.log(g)
            else:
                lo = math.log(g)
        print(f"MID_POINTS[({arch.B}, {arch.N}, {arch.M})] = ({g:.4f}, {s:.4f})  # {bpp:.3f} bpp on {SIZE}x{SIZE} noise")


if __name__ == "__main__":
    main()
