#!/usr/bin/env python3
"""Team decoder experiment: decode time of T = 1, 2, 4, 8 batches of 32 B8_lowrate 768x768 frames in one
k_dec_team launch against the graph decoder (one batch per lbc_decode call), and the per-operation barrier
stamps of one sampled raster step.  Prints one JSON line per measurement."""
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
from lbic.model import BlockBasedImgCompLossyNetv9, decompress_teams  # noqa: E402
from lbic.weights import synth_state_dict  # noqa: E402


CONFIGS = {   # name -> (B, KS, N, M, synthetic-weight operating point of the config: bench.py / lbic.weights)
    "B8_lowrate": (8, (3, 1, 1, 1), 768, 96, "low"),
    "B8_highrate": (8, (3, 3, 1, 1), 1152, 128, "mid"),
    "B4_highrate": (4, (3, 3, 1, 1), 512, 96, "mid"),
    "B16_lowrate": (16, (3, 1, 1, 1), 1280, 192, "low"),
}


def main():
    # CONFIG / SIZE / HEIGHT / BATCH: the frames of one batch; TB: batches per team (a team decodes TB x BATCH images,
    # the bench's --team-batches); TEAMS: comma-separated team counts per launch; ONE=1: one launch per team count
    # (no untimed warm launch: PMC passes)
    B, KS, N, M, rate = CONFIGS[os.environ.get("CONFIG", "B8_lowrate")]
    size = int(os.environ.get("SIZE", "768"))
    height = int(os.environ.get("HEIGHT", "0")) or size
    n = int(os.environ.get("BATCH", "32"))
    tb = int(os.environ.get("TB", "1"))
    Ts = [int(t) for t in os.environ.get("TEAMS", "1,2,4,8").split(",")]
    arch = Arch(B, KS, N, M)
    cfg = types.SimpleNamespace(block_size=B, KS=list(KS), N=N, M=M, gpu_device=0)
    m = BlockBasedImgCompLossyNetv9(cfg)
    m.load_state_dict(synth_state_dict(arch, 1337, rate=os.environ.get("RATE", rate)))
    m.update(force=True)
    hs = [m] + [m.sibling() for _ in range(max(Ts) - 1)]
    Hb, Wb = height // B, size // B
    fr = np.stack([image_to_blocks(np.random.default_rng(k).integers(0, 256, (3, height, size), dtype=np.uint8)
                                   .astype(np.float32) / 255.0 - 0.5, B) for k in range(n)])
    x = torch.from_numpy(fr).cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    print(json.dumps(dict(bpp=float(np.mean([len(s) * 8.0 / (size * height) for s in st])))), flush=True)
    if tb > 1:      # a team's images: tb copies of the batch side by side
        st = st * tb
        r = {"zhat": torch.cat([r["zhat"]] * tb)}
    if not os.environ.get("SKIP_GRAPH"):
        z = m.decompress_batch(st, Hb, Wb)
        assert torch.equal(z, r["zhat"])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        z = m.decompress_batch(st, Hb, Wb)
        torch.cuda.synchronize()
        tg = time.perf_counter() - t0
        print(json.dumps(dict(decoder="graph", batches=1, seconds=round(tg, 4), ms_per_batch=round(tg * 1e3, 2))),
              flush=True)
    for T in Ts:
        tsz = int(os.environ.get("TEAM_SIZE", "0"))
        ok = None
        if not os.environ.get("ONE"):
            zs = decompress_teams(hs, [st] * T, Hb, Wb, wg_per_cu=int(os.environ.get("WPC", "1")), team_size=tsz)  # warm
            ok = all(torch.equal(zz, r["zhat"]) for zz in zs)
        os.environ["LBIC_TEAM_STAMPS"] = "1"
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        zs = decompress_teams(hs, [st] * T, Hb, Wb, wg_per_cu=int(os.environ.get("WPC", "1")), team_size=tsz)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        os.environ["LBIC_TEAM_STAMPS"] = "0"
        if ok is None:
            ok = all(torch.equal(zz, r["zhat"]) for zz in zs)
        ts = hs[0].team_stamps()
        if len(ts[0]) < 1024 or Hb < 2 or Wb < 2:
            print(json.dumps(dict(decoder="team", batches=T, seconds=round(dt, 4), ms_per_batch=round(dt * 1e3 / T, 2),
                                  bit_exact=ok, mode=hs[0].team_stats()["mode"])), flush=True)
            continue
        ops, comp = [], []
        for row in ts:
            prev = row[60]
            d, c = [], []
            for k in range(12):
                d.append(round((row[k] - prev) / 100.0, 2))      # us (100 MHz): op start -> past its barrier
                c.append(round((row[32 + k] - prev) / 100.0, 2))  # op start -> team rank 0's own work done
                prev = row[k]
            ops.append(d)
            comp.append(c)
        if os.environ.get("RAW_OUT"):      # every team's raw stamp block (offline decomposition)
            with open(os.environ["RAW_OUT"] + f"_T{T}.json", "w") as f:
                json.dump([[int(v) for v in row] for row in ts], f)
        span = [round((row[63] - row[62]) / 1e5, 2) for row in ts]
        step = [round((row[61] - row[60]) / 100.0, 2) for row in ts]
        print(json.dumps(dict(decoder="team", batches=T, seconds=round(dt, 4), ms_per_batch=round(dt * 1e3 / T, 2),
                              bit_exact=ok, launch_ms=span, sampled_step_us=step, op_us_team0=ops[0],
                              op_us_mean=[round(float(np.mean([o[k] for o in ops])), 2) for k in range(12)],
                              work_us_team0=comp[0], sc1=os.environ.get("LBIC_TEAM_SC1", "0"),
                              rans_done_us=[round((ts[0][160 + k] - ts[0][3]) / 100.0, 2) if ts[0][160 + k] else None
                                            for k in range(32)],
                              gemm_beside_rans_done_us=[round((ts[0][192 + k] - ts[0][3]) / 100.0, 2) if ts[0][192 + k]
                                                        else None for k in range(32)],
                              intra_cycles_team0=[[ts[0][256 + 64 * k + p] - ts[0][256 + 64 * k] if ts[0][256 + 64 * k + p] else 0
                                                   for p in range(1, 48)] for k in range(12)])),
              flush=True)


if __name__ == "__main__":
    main()
