"""Summarise a rocprofv3 --kernel-trace --stats CSV (run_kernel_stats.csv) per kernel family.

usage: python tools/kstats_summary.py kernel_stats.csv [kernel_trace.csv]
Prints, per family (template arguments dropped: k_gemm_s, k_gemm, k_rans_decode, ...), the call count, the
total and the average dispatch-to-completion duration in microseconds over the whole command; with the
kernel trace also the same table for the dispatches inside bench.py's timed region (between its two
spin_kernel markers) -- the figures bench.py's roofline (avg_launch_us of the dominant family) must agree with -- and
each family's wall occupancy there (the union of its launches' intervals: bench.py's dominance rule).
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


def region(path):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        return
    kn = next(k for k in rows[0] if "Name" in k and "Kernel" in k)
    ks = next(k for k in rows[0] if "Start" in k)
    ke = next(k for k in rows[0] if "End" in k)
    spins = sorted((int(r[ks]), int(r[ke])) for r in rows if "spin_kernel" in r[kn])
    if len(spins) < 2:
        print("(no timed-region markers in the trace)")
        return
    t0, t1 = spins[0][1], spins[-1][0]
    fam = defaultdict(lambda: [0, 0.0])
    spans = defaultdict(list)
    for r in rows:
        s_, e_ = int(r[ks]), int(r[ke])
        if t0 <= s_ and e_ <= t1 and "spin_kernel" not in r[kn]:
            f = family(r[kn])
            fam[f][0] += 1
            fam[f][1] += e_ - s_
            spans[f].append((s_, e_))

    def union(iv):          # wall occupancy: the time at least one launch of the set is running
        tot, cur_s, cur_e = 0, None, None
        for s_, e_ in sorted(iv):
            if cur_e is None or s_ > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s_, e_
            else:
                cur_e = max(cur_e, e_)
        return tot + (cur_e - cur_s if cur_e is not None else 0)
    print(f"\ntimed region only ({(t1 - t0) / 1e9:.3f} s between the markers)")
    print(f"{'family':32s} {'calls':>10s} {'total_ms':>10s} {'avg_us':>8s} {'occupancy_ms':>12s}")
    for f, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{f:32s} {c:10d} {t / 1e6:10.2f} {t / c / 1e3:8.3f} {union(spans[f]) / 1e6:12.2f}")
    enc = [iv for f in ("k_gemm", "k_gemm_s") for iv in spans.get(f, [])]
    if enc:
        print(f"{'encoder GEMMs (k_gemm + k_gemm_s)':32s} {len(enc):10d} {sum(e - s for s, e in enc) / 1e6:10.2f} "
              f"{'':8s} {union(enc) / 1e6:12.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
    if len(sys.argv) > 2:
        region(sys.argv[2])
