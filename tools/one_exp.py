#!/usr/bin/env python3
"""Single-image decode experiment (k_dec_one, csrc/one.hip): one seeded 768x768 B8_lowrate frame encoded by the
library, decoded through lbc_decode as one image -- k_dec_one -- and through the row graphs (LBIC_ONE=0), host clock
around synchronize (eval_model's timing), median of REPS; then one decode with LBIC_ONE_STAMPS=1: per-operation stamps
of the middle raster step.  Prints JSON lines."""
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "learned-block-based-image-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lbic.arch import Arch  # noqa: E402
from lbic.layout import image_to_blocks  # noqa: E402
from lbic.model import BlockBasedImgCompLossyNetv9  # noqa: E402
from lbic.weights import synth_state_dict  # noqa: E402

OPS = ["ctx0", "ctx1", "ctx2", "ctx3", "rans", "dec0", "ig0", "d1", "ig1", "d2", "ig2", "d3", "rans_idx_coded"]


CONFIGS = {   # name -> (B, KS, N, M, synthetic-weight operating point of the config: bench.py / lbic.weights)
    "B8_lowrate": (8, (3, 1, 1, 1), 768, 96, "low"),
    "B4_highrate": (4, (3, 3, 1, 1), 512, 96, "mid"),
}


def main():
    # CONFIG: B8_lowrate (default) or B4_highrate (KS3311: layer-0 cache, half-tile layer 1); SIZE: frame side
    B, KS, N, M, rate = CONFIGS[os.environ.get("CONFIG", "B8_lowrate")]
    size = int(os.environ.get("SIZE", "768"))
    reps = int(os.environ.get("REPS", "3"))
    arch = Arch(B, KS, N, M)
    cfg = types.SimpleNamespace(block_size=B, KS=list(KS), N=N, M=M, gpu_device=0)
    m = BlockBasedImgCompLossyNetv9(cfg)
    m.load_state_dict(synth_state_dict(arch, 1337, rate=os.environ.get("RATE", rate)))
    m.update(force=True)
    img = np.random.default_rng(12345).integers(0, 256, (3, size, size), dtype=np.uint8).astype(np.float32) / 255 - 0.5
    x = torch.from_numpy(image_to_blocks(img, B))[None].cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    print(json.dumps(dict(config=os.environ.get("CONFIG", "B8_lowrate"), bpp=len(st[0]) * 8.0 / (size * size))),
          flush=True)
    Hb = Wb = size // B
    for mode in ("1", "0"):
        os.environ["LBIC_ONE"] = mode
        ts = []
        for k in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.time()
            z = m.decompress_batch(st, Hb, Wb)
            torch.cuda.synchronize()
            if k:
                ts.append(time.time() - t0)
        print(json.dumps(dict(decoder=m.decode_path()["path"], ms=round(float(np.median(ts)) * 1e3, 2),
                              us_per_step=round(float(np.median(ts)) * 1e6 / (Hb * Wb), 2),
                              bit_exact=bool(torch.equal(z, r["zhat"])))), flush=True)
    os.environ["LBIC_ONE"] = "1"
    os.environ["LBIC_ONE_STAMPS"] = "1"
    z = m.decompress_batch(st, Hb, Wb)
    os.environ["LBIC_ONE_STAMPS"] = "0"
    s = m.one_stamps()
    print(json.dumps(dict(stamps_us={OPS[o]: s[o] for o in range(len(s))}, bit_exact=bool(torch.equal(z, r["zhat"])))),
          flush=True)
    d = m.one_phase_stamps()
    print(json.dumps(dict(phases_us={OPS[o]: d[o] for o in range(len(d))},
                          keys=["in", "first_ready", "last_ready", "regs", "chain", "reduced", "stored", "published", "ready_by_wave"])), flush=True)


if __name__ == "__main__":
    main()
