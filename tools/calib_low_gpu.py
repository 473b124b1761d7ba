#!/usr/bin/env python3
"""Calibrate lbic.weights.LOW_POINTS for B16_lowrate at the bench's own frames: bisection on the
latent gain of rate="low" so that the seeded 2048x2048 noise frames bench.py codes for config 5 (default_rng(k), k =
0, 1) average the config's published 0.120 bpp (experiments/blkbsdimgcomp_B16_KS3111_N1280M192_v9/
exp_117.045/logs/exp_debug.log:930-955).  Runs the product library on the GPU (compress + host rANS); prints one JSON
line per probe and the LOW_POINTS entry.

    python tools/calib_low_gpu.py [target] [size]
"""
import json
import math
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "learned-block-based-image-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lbic.arch import Arch  # noqa: E402
from lbic.layout import image_to_blocks  # noqa: E402
from lbic.model import BlockBasedImgCompLossyNetv9  # noqa: E402
from lbic.weights import synth_state_dict  # noqa: E402


def main():
    target = float(sys.argv[1]) if len(sys.argv) > 1 else 0.120
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    arch = Arch(16, (3, 1, 1, 1), 1280, 192)
    cfg = types.SimpleNamespace(block_size=16, KS=[3, 1, 1, 1], N=1280, M=192, gpu_device=0)
    fr = np.stack([image_to_blocks(np.random.default_rng(k).integers(0, 256, (3, size, size), dtype=np.uint8)
                                   .astype(np.float32) / 255.0 - 0.5, 16) for k in range(2)])
    x = torch.from_numpy(fr).cuda()
    lo, hi = math.log(0.2), math.log(1.0)
    g = bpp = None
    for it in range(9):
        g = math.exp(0.5 * (lo + hi))
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(synth_state_dict(arch, 1337, rate="low", mid=(g, 0.0)))
        m.update(force=True)
        r = m.compress_batch(x)
        st = m.entropy_encode(r["symbols"], r["indexes"])
        bpp = float(np.mean([len(s) * 8.0 / size ** 2 for s in st]))
        print(json.dumps(dict(gain=round(g, 5), bpp=round(bpp, 5), target=target)), flush=True)
        del m, r
        torch.cuda.empty_cache()
        if bpp > target:
            hi = math.log(g)
        else:
            lo = math.log(g)
    print(f"LOW_POINTS[(16, 1280, 192)] = {g:.4f}  # {bpp:.4f} bpp on the bench's {size}x{size} noise frames", flush=True)


if __name__ == "__main__":
    main()
