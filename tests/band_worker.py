"""Worker of tests/test_band_gpu.py (launched with torch.distributed.run, gloo, every rank on cuda:0 of a one-GPU
box): codes seeded frames split into bands over the ranks (lbic.band) and has rank 0 save the gathered band
results.  Cases: (a) KS3311 tiny geometry, 3 bands over 5 block rows (2, 2, 1 rows: a one-row band forwards its
halo), chunks of 3 steps; (b) B8_lowrate geometry, 2 bands (ranks 0, 1) over 6 block rows, chunks of 1 step."""
import argparse
import os
import sys
import types

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learned-block-based-image-compression_amd"))
from lbic.arch import Arch  # noqa: E402
from lbic.band import band_rows, compress_band, gather_bands  # noqa: E402
from lbic.model import BlockBasedImgCompLossyNetv9  # noqa: E402
from lbic.weights import synth_state_dict  # noqa: E402

CASES = {   # name -> (arch, Hb, Wb, n_img, bands, chunk)
    "ks3311_3bands": (Arch(4, (3, 3, 1, 1), 64, 16), 5, 12, 2, 3, 3),
    "b8_lowrate_2bands": (Arch(8, (3, 1, 1, 1), 768, 96), 6, 16, 2, 2, 1),
}


def frames(arch, Hb, Wb, n, seed):
    rng = np.random.default_rng(seed)
    return (rng.integers(0, 256, (n, Hb, Wb, arch.cx)).astype(np.float32) / 255.0 - 0.5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    res = {}
    for name, (arch, Hb, Wb, n, P, chunk) in CASES.items():
        group = dist.new_group(list(range(P)))
        if rank >= P:
            continue
        cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
        m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
        m.load_state_dict(synth_state_dict(arch, 1337))
        m.update(force=True)
        x = frames(arch, Hb, Wb, n, 9)
        v0, rows = band_rows(Hb, P)[rank]
        part = compress_band(m, torch.from_numpy(x[:, v0:v0 + rows]).to(dev), v0, Hb, group=group, chunk=chunk,
                             transport="host")
        full = gather_bands(part, group=group)
        if rank == 0:
            for k, v in full.items():
                res[f"{name}/{k}"] = v.cpu().numpy()
    dist.barrier()
    if rank == 0:
        np.savez(a.out, **res)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
