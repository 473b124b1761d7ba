"""Merge the PMC passes of tools/pmc_configs.sh into per-config traffic entries for bench.py (profiles/pmc_traffic.json
"configs"): per config, the team decoder's fabric bytes per batch raster step (one --batch batch, one raster step) at
the config's own launch shape, and the encoder graph's bytes per k_gemm / k_gemm_s dispatch.

usage: python tools/pmc_configs.py OUT.json DIR     (DIR: gpurun_out/pmc_cfg)
"""
import json
import os
import sys

SHAPES = {   # tag -> (teams, batches per team, frames per batch, Hb, Wb, description): tools/pmc_configs.sh
    "B8_highrate": (8, 2, 3, 64, 96, "8 teams of 2 x 3 frames of 768x512 (64 x 96 blocks of 8x8) per dispatch"),
    "B4_highrate": (16, 1, 32, 192, 192, "16 teams of 32 frames of 768x768 (192 x 192 blocks of 4x4) per dispatch"),
    "B16_lowrate": (8, 2, 8, 128, 128, "8 teams of 2 x 8 frames of 2048x2048 (128 x 128 blocks of 16x16) per dispatch"),
}


def main():
    out, d = sys.argv[1], sys.argv[2]
    res = {}
    for tag, (T, tb, n, Hb, Wb, desc) in SHAPES.items():
        tf, ef = os.path.join(d, tag + "_team.json"), os.path.join(d, tag + "_enc.json")
        if not (os.path.exists(tf) and os.path.exists(ef)):
            continue
        team, enc = json.load(open(tf)), json.load(open(ef))
        e = {}
        if "k_dec_team" in team and "hbm_bytes_per_dispatch" in team["k_dec_team"]:
            t = dict(team["k_dec_team"])
            t["hbm_bytes_per_batch_step"] = t["hbm_bytes_per_dispatch"] / (T * tb * Hb * Wb)
            t["source"] = f"tools/team_exp.py under FETCH_SIZE / WRITE_SIZE passes (tools/pmc_configs.sh): {desc}"
            e["k_dec_team"] = t
        for k in ("k_gemm", "k_gemm_s"):
            if k in enc and "hbm_bytes_per_dispatch" in enc[k]:
                e[k] = dict(dispatches=enc[k]["dispatches"], hbm_bytes_per_dispatch=enc[k]["hbm_bytes_per_dispatch"],
                            source=f"tools/enc_exp.py under FETCH_SIZE / WRITE_SIZE passes: the {tag} encoder graph of "
                                   f"one wavefront pass of 4 batches of {n} frames (bench --enc-pass 4)")
        res[tag] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
