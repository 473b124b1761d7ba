#!/usr/bin/env python3
"""Encoder experiment: compress time of one batch of 32 B8_lowrate 768x768 frames (encoder alone, HIP events around
the wavefront graph), and a digest of its symbols / indexes / zhat to compare kernel variants (LBIC_ENC_TILED ...)."""
import hashlib
import json
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


CONFIGS = {   # name -> (B, KS, N, M, synthetic-weight operating point of the config: bench.py / lbic.weights)
    "B8_lowrate": (8, (3, 1, 1, 1), 768, 96, "low"),
    "B8_highrate": (8, (3, 3, 1, 1), 1152, 128, "mid"),
    "B4_highrate": (4, (3, 3, 1, 1), 512, 96, "mid"),
    "B16_lowrate": (16, (3, 1, 1, 1), 1280, 192, "low"),
}


def main():
    B, KS, N, M, rate = CONFIGS[os.environ.get("CONFIG", "B8_lowrate")]
    size = int(os.environ.get("SIZE", "768"))
    height = int(os.environ.get("HEIGHT", "0")) or size
    n = int(os.environ.get("BATCH", "32"))
    arch = Arch(B, KS, N, M)
    cfg = types.SimpleNamespace(block_size=B, KS=list(KS), N=N, M=M, gpu_device=0)
    m = BlockBasedImgCompLossyNetv9(cfg)
    m.load_state_dict(synth_state_dict(arch, 1337, rate=os.environ.get("RATE", rate)))
    m.update(force=True)
    if os.environ.get("LDS_FLOOR"):
        m.set_encoder_lds_floor(int(os.environ["LDS_FLOOR"]))
    fr = np.stack([image_to_blocks(np.random.default_rng(k).integers(0, 256, (3, height, size), dtype=np.uint8)
                                   .astype(np.float32) / 255.0 - 0.5, B) for k in range(n)])
    x = torch.from_numpy(fr).cuda()
    r = m.compress_batch(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(int(os.environ.get("REPS", "3"))):
        r = m.compress_batch(x)
        torch.cuda.synchronize()
        ts.append(m.last_timing()[0])
    h = hashlib.sha256()
    for k in ("symbols", "indexes", "zhat"):
        h.update(r[k].cpu().numpy().tobytes())
    print(json.dumps(dict(config=os.environ.get("CONFIG", "B8_lowrate"), batch=n, lds_floor=os.environ.get("LDS_FLOOR", "0"), encode_ms=[round(t, 2) for t in ts],
                          digest=h.hexdigest()[:16])), flush=True)


if __name__ == "__main__":
    main()
