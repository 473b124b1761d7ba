"""Build profiles/pmc_traffic.json (read by bench.py for roofline.traffic) from PMC passes at the headline's shapes.

usage: python tools/pmc_headline.py OUT.json ENC.json TEAM.json [teams Hb Wb images_per_team]
ENC.json: tools/pmc_summary.py over FETCH_SIZE / WRITE_SIZE passes of tools/enc_exp.py (one 32-frame B8_lowrate
768x768 batch per compression: exactly the encoder graph the bench replays), per kernel (k_gemm_t / k_gemm /
k_gemm_s) and as the graph's dispatch-weighted mean.  TEAM.json: tools/pmc_summary.py over the FETCH_SIZE / WRITE_SIZE / TCC passes of
tools/team_exp.py (8 teams per k_dec_team launch); per team raster step = per dispatch / (teams x Hb x Wb), per
32-frame batch step (what bench.py scales by the batches a launch decodes) = per dispatch / (teams x images / 32 x Hb x Wb).
"""
import json
import os
import sys


def main():
    out, encf, teamf = sys.argv[1:4]
    T, Hb, Wb, nimg = (int(x) for x in (sys.argv[4:8] if len(sys.argv) > 7 else (8, 96, 96, 32)))
    enc, team = json.load(open(encf)), json.load(open(teamf))
    res = {}
    z = {"dispatches": 0, "hbm_bytes_per_dispatch": 0.0}
    # per kernel of the encoder graph (k_gemm_t: the wide layers; k_gemm: the narrow ones, or all when k_gemm_t is
    # off; k_gemm_s: the wavefront's ramp steps), and the graph's dispatch-weighted mean under the bench's family name
    for k in ("k_gemm_t", "k_gemm", "k_gemm_s"):
        if k in enc:
            res[k] = dict(dispatches=enc[k]["dispatches"], hbm_bytes_per_dispatch=enc[k]["hbm_bytes_per_dispatch"],
                          source="tools/enc_exp.py under FETCH_SIZE / WRITE_SIZE passes: the encoder graph of one "
                                 f"{os.environ.get('BATCH', '32')}-frame 768x768 B8_lowrate wavefront pass")
    fams = [enc.get(k, z) for k in ("k_gemm_t", "k_gemm", "k_gemm_s")]
    n = sum(f["dispatches"] for f in fams)
    res["encoder_graph"] = dict(dispatches=n, hbm_bytes_per_dispatch=sum(f["hbm_bytes_per_dispatch"] * f["dispatches"]
                                                                        for f in fams) / max(n, 1),
                                source="every dispatch of the encoder graph, dispatch-weighted")
    t = dict(team["k_dec_team"])
    t["hbm_bytes_per_team_step"] = t["hbm_bytes_per_dispatch"] / (T * Hb * Wb)
    t["hbm_bytes_per_batch_step"] = t["hbm_bytes_per_dispatch"] / (T * nimg / 32 * Hb * Wb)
    t["images_per_team"] = nimg
    if "TCC_HIT_sum" in t:
        t["l2_hit_rate"] = t["TCC_HIT_sum"] / (t["TCC_HIT_sum"] + t["TCC_MISS_sum"])
    t["source"] = f"tools/team_exp.py under PMC passes: {T} teams of {nimg} images x {Hb}x{Wb} blocks per dispatch"
    res["k_dec_team"] = t
    res["_source"] = {"note": "FETCH_SIZE x 2 + WRITE_SIZE, x 1024 bytes (MI355X_MICROARCH.md HBM section)"}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
