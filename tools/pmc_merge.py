"""Merge the team decoder's PMC passes (tools/team_pmc.sh: 8 batches of 32 B8_lowrate 768x768 frames per k_dec_team
launch) into the headline's PMC file (tools/gpu_profile.sh: the encoder's launch shapes), per team raster step.

usage: python tools/pmc_merge.py pmc_traffic.json team_pmc.json OUT.json [teams Hb Wb]
k_dec_team's per-dispatch bytes are divided by teams x Hb x Wb (defaults 8 x 96 x 96) into hbm_bytes_per_team_step,
which bench.py scales by the team-steps of its own launches (the gpu_profile run's k_dec_team entry codes 64x64
frames and is replaced).
"""
import json
import sys


def main():
    base, team, out = sys.argv[1:4]
    T, Hb, Wb = (int(x) for x in (sys.argv[4:7] if len(sys.argv) > 6 else (8, 96, 96)))
    p = json.load(open(base))
    t = json.load(open(team))["k_dec_team"]
    steps = T * Hb * Wb
    t = dict(t)
    t["hbm_bytes_per_team_step"] = t["hbm_bytes_per_dispatch"] / steps
    t["l2_hit_rate"] = t["TCC_HIT_sum"] / (t["TCC_HIT_sum"] + t["TCC_MISS_sum"])
    t["source"] = f"tools/team_pmc.sh: {T} batches x {Hb}x{Wb} blocks per dispatch"
    p["k_dec_team"] = t
    json.dump(p, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main()
