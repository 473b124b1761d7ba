#!/usr/bin/env python3
"""Per-shape encoder launch times from a rocprofv3 kernel trace of tools/enc_exp.py: k_gemm dispatches grouped by
their grid (N tiles x M tiles), with count, mean duration and the share of the encoder's total kernel time.

usage: python tools/enc_shapes.py kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    acc = defaultdict(list)
    tot = 0.0
    with open(sys.argv[1]) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "")
            if "k_gemm" not in name:
                continue
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
            gy = int(r.get("Grid_Size_Y", 1) or 1)
            fam = "k_gemm_s" if "k_gemm_s" in name else "k_gemm_t" if "k_gemm_t" in name else "k_gemm"
            acc[(fam, gx // max(wx, 1), gy)].append(d)
            tot += d
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    print(f"total k_gemm* kernel time {tot / 1e3:.2f} ms over {sum(len(v) for v in acc.values())} dispatches")
    print("family  grid_x(N tiles) grid_y(M tiles)  count  mean_us  share")
    for (fam, gx, gy), v in rows[:40]:
        print(f"{fam:8s} {gx:6d} {gy:6d} {len(v):7d} {sum(v) / len(v):8.2f} {sum(v) / tot:6.3f}")


if __name__ == "__main__":
    main()
