"""Summarise a rocprofv3 --kernel-trace --stats CSV (run_kernel_stats.csv) per kernel family.

usage: python tools/kstats_summary.py kernel_stats.csv
Prints, per family (template arguments dropped: k_gemm_s, k_gemm, k_rans_decode, ...), the call count, the
total and the average dispatch-to-completion duration in microseconds -- the figures bench.py's roofline
(avg_launch_us of the dominant family) must agree with.
"""
import csv
import re
import sys
from collections import defaultdict


def family(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    name = name.replace("lbic::", "")
    return re.sub(r"<.*>$", "", name).strip()


def main(path):
    fam = defaultdict(lambda: [0, 0.0])
    for row in csv.DictReader(open(path)):
        f = family(row["Name"])
        fam[f][0] += int(row["Calls"])
        fam[f][1] += float(row["TotalDurationNs"])
    print(f"{'family':32s} {'calls':>10s} {'total_ms':>10s} {'avg_us':>8s}")
    for f, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{f:32s} {c:10d} {t / 1e6:10.2f} {t / c / 1e3:8.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
