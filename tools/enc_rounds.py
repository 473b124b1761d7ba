"""Encoder launch accounting from a rocprofv3 --kernel-trace of tools/enc_exp.py: per k_gemm
shape (N columns, M rows from the grid), workgroups against the resident slots, rounds, the average duration and the
time per round; the gap between consecutive dispatches of one queue; and the graph's timeline split into dispatch time
and launch gaps.

usage: python tools/enc_rounds.py TRACE_DIR [slots]
slots: resident k_gemm workgroups on the chip (default 1024 = 256 CUs x 4: 60 VGPRs -> 8 waves per SIMD, 8 waves per
workgroup; 16 KB of LDS each).  k_gemm<16,32,8,1>: grid = (N/32 x 512 threads, M/16); k_gemm_s: (N/16 x 512, M/16).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("lbic::", ""))
            if not name.startswith("k_gemm"):
                continue
            gx, gy = int(r["Grid_Size_X"]), int(r["Grid_Size_Y"])
            wx = int(r["Workgroup_Size_X"])
            rows.append(dict(s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"]), k=name, q=r.get("Queue_Id", ""),
                             wg=(gx // wx) * gy, N=(gx // wx) * (32 if name.startswith("k_gemm<") else 16), M=gy * 16))
    rows.sort(key=lambda r: r["s"])
    # the last compress of the run (enc_exp.py: one capture pass + REPS timed passes): dispatches after the largest gap
    big = max(range(1, len(rows)), key=lambda i: rows[i]["s"] - rows[i - 1]["e"])
    last = rows[big:] if len(rows) - big > 1000 else rows
    shapes = defaultdict(list)
    for r in last:
        shapes[(r["k"], r["N"], r["wg"] // 64 * 64)].append(r)
    out = []
    for (k, N, wgb), v in sorted(shapes.items(), key=lambda kv: -sum(x["e"] - x["s"] for x in kv[1])):
        dur = sum(x["e"] - x["s"] for x in v) / len(v) / 1e3
        wg = sum(x["wg"] for x in v) / len(v)
        rounds = wg / slots
        out.append(dict(kernel=k, N=N, workgroups=round(wg), rounds=round(rounds, 2), dispatches=len(v),
                        mean_us=round(dur, 2), us_per_full_round=round(dur / max(1.0, -(-wg // slots)), 2),
                        total_ms=round(dur * len(v) / 1e3, 2)))
    span = (last[-1]["e"] - last[0]["s"]) / 1e6
    busy = 0.0      # union of dispatch intervals
    cur_s, cur_e = None, None
    for r in last:
        if cur_e is None or r["s"] > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = r["s"], r["e"]
        else:
            cur_e = max(cur_e, r["e"])
    busy += cur_e - cur_s
    gaps = defaultdict(list)
    prevq = {}
    for r in last:
        p = prevq.get(r["q"])
        if p is not None and r["s"] >= p["e"]:
            gaps[r["q"]].append((r["s"] - p["e"]) / 1e3)
        prevq[r["q"]] = r
    res = dict(dispatches=len(last), graph_span_ms=round(span, 3), any_dispatch_running_ms=round(busy / 1e6, 3),
               idle_ms=round(span - busy / 1e6, 3),
               queue_gaps_us={q: dict(n=len(g), mean=round(sum(g) / len(g), 2), median=round(sorted(g)[len(g) // 2], 2))
                              for q, g in gaps.items() if g},
               slots=slots, shapes=out)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
