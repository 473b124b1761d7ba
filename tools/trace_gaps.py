"""Per-kernel durations and the gaps between consecutive kernels of one stream from a rocprofv3
--kernel-trace CSV (decode phase of a small bench run).  usage: python tools/trace_gaps.py DIR"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
rows.sort()
name = lambda k: re.sub(r"\(.*", "", k.replace("void ", "").replace("lbic::", ""))
# the raster decoder's kernels: the longest run of k_gemm_s / k_rans_decode in one queue
dur = defaultdict(list)
gap = defaultdict(list)
prev = None
for s, e, k, q in rows:
    n = name(k)
    dur[n].append((e - s) / 1e3)
    if prev is not None and prev[3] == q and 0 <= s - prev[1] < 50_000:
        gap[(name(prev[2]), n)].append((s - prev[1]) / 1e3)
    prev = (s, e, k, q)
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{n:32s} n={len(v):7d} mean {sum(v)/len(v):8.2f} us  median {v[len(v)//2]:8.2f}")
print("gaps (us) between consecutive kernels on one queue:")
for k, v in sorted(gap.items(), key=lambda kv: -len(kv[1]))[:12]:
    v.sort()
    print(f"  {k[0]:26s} -> {k[1]:26s} n={len(v):7d} mean {sum(v)/len(v):6.2f} median {v[len(v)//2]:6.2f}")
