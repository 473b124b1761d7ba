"""Timeline summary of a rocprofv3 --kernel-trace CSV: over the middle part of the trace (--lo/--hi fractions of its
span, default 0.25..0.75: the steady state of a pipelined bench run), the fraction of time with >= 1 kernel running,
the time-weighted mean number of kernels in flight, per kernel family the count and mean duration, and per queue
its busy fraction and the gap between a kernel's end and the next kernel's start on that queue (the launch boundary
as the hardware sees it).  usage: python tools/trace_timeline.py DIR [--lo F] [--hi F]"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--lo", type=float, default=0.25)
ap.add_argument("--hi", type=float, default=0.75)
a = ap.parse_args()
f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = []
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
rows.sort()
t0, t1 = rows[0][0], max(r[1] for r in rows)
lo, hi = t0 + a.lo * (t1 - t0), t0 + a.hi * (t1 - t0)
win = [r for r in rows if r[0] >= lo and r[1] <= hi]
span = hi - lo
name = lambda k: re.sub(r"[<(].*", "", k.replace("void ", "").replace("lbic::", ""))
ev = []
for s, e, _, _ in win:
    ev.append((s, 1))
    ev.append((e, -1))
ev.sort()
busy = 0
area = 0
cur = 0
last = lo
for t, d in ev:
    if cur > 0:
        busy += t - last
    area += cur * (t - last)
    cur += d
    last = t
print(f"window {span / 1e6:.1f} ms of {(t1 - t0) / 1e6:.1f} ms, {len(win)} kernels ({len(win) / span * 1e9 / 1e3:.0f} k/s)")
print(f"GPU busy (>= 1 kernel) {busy / span:.3f} of the window; mean kernels in flight {area / span:.2f}")
fam = defaultdict(list)
for s, e, k, _ in win:
    fam[name(k)].append((e - s) / 1e3)
for n, v in sorted(fam.items(), key=lambda kv: -sum(kv[1]))[:8]:
    v.sort()
    print(f"  {n:28s} n={len(v):7d} mean {sum(v) / len(v):7.2f} us median {v[len(v) // 2]:7.2f} "
          f"sum {sum(v) / 1e3:8.1f} ms")
byq = defaultdict(list)
for r in win:
    byq[r[3]].append(r)
print("per queue: kernels, busy fraction, end->next start gap mean / median (us), dominant kernel")
for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    rs.sort()
    b = sum(e - s for s, e, _, _ in rs)
    gaps = sorted((rs[i + 1][0] - rs[i][1]) / 1e3 for i in range(len(rs) - 1) if rs[i + 1][0] >= rs[i][1])
    dom = max(set(name(k) for _, _, k, _ in rs), key=lambda n: sum(1 for _, _, k, _ in rs if name(k) == n))
    if gaps:
        print(f"  queue {q:>4s}: {len(rs):7d}  busy {b / span:.3f}  gap mean {sum(gaps) / len(gaps):7.2f} "
              f"median {gaps[len(gaps) // 2]:6.2f}  ({dom})")
