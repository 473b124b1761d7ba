#!/usr/bin/env python3
"""Per-operation decomposition of one k_dec_team raster step from a tools/team_exp.py log of the
diagnostic build (make team_diag, LBIC_LIB_VARIANT=tdiag): team rank 0's shader-clock stamps (team.hip dstamp) of the
sampled step, per operation, converted to microseconds with the operation's own clock rate (its stamped cycles over
its s_memrealtime work time).  Columns:
  prologue   entry -> every A-fragment load issued (wave 0): epilogue operands (bias / GDN input), first weight
             fragments, A addressing
  first A    loads issued -> the slowest wave's first A fragment in registers (memory latency of the hand-off data)
  chains     first A -> the slowest wave's last chain done (MFMA chains of every item, next-item weights in flight)
  reduce+epi workgroup barrier -> outputs written (partials summed in slice order, epilogue, stores issued)
  drain+sync outputs written -> past the team barrier (store drain vmcnt(0), one arrival per workgroup, the poll)
usage: python tools/team_ops_table.py LOG [--md]
"""
import json
import sys

OPS = ["ctx0", "ctx1", "ctx2", "ctx3", "rANS", "dec0", "igdn0", "dec1", "igdn1", "dec2", "igdn2", "dec3"]


def main():
    path = sys.argv[1]
    md = "--md" in sys.argv
    d = None
    for line in open(path):
        if line.startswith('{"decoder": "team"'):
            d = json.loads(line)
    rows = []
    for k, cyc in enumerate(d["intra_cycles_team0"]):
        op, work = d["op_us_team0"][k], d["work_us_team0"][k]
        if not any(cyc) or not cyc[3]:
            rows.append((OPS[k], op, work, None))
            continue
        f = cyc[3] / work          # cycles per us (p4 = outputs written ~ the op's work end)
        p = lambda i: cyc[i - 1] / f if i >= 1 and cyc[i - 1] else 0.0    # stamp p (1-based list: index p - 1)
        issued = p(1)
        first_a = max(cyc[39:47]) / f if any(cyc[39:47]) else issued
        last_chain = max(cyc[15:23]) / f if any(cyc[15:23]) else p(3)
        bar = p(8)
        out = p(4)
        rows.append((OPS[k], op, work, dict(prologue=issued, first_a=max(0.0, first_a - issued),
                                             chains=max(0.0, last_chain - first_a), wg_bar=max(0.0, bar - last_chain),
                                             reduce_epi=max(0.0, out - bar), drain_sync=max(0.0, op - out),
                                             mhz=f)))
    hdr = ["op", "op us", "prologue", "first A", "chains", "wg barrier", "reduce+epi", "drain+sync"]
    if md:
        print("| " + " | ".join(hdr) + " |")
        print("|" + "---|" * len(hdr))
    tot = [0.0] * 7
    for name, op, work, r in rows:
        if r is None:
            vals = [op, None, None, None, None, None, op - work]
        else:
            vals = [op, r["prologue"], r["first_a"], r["chains"], r["wg_bar"], r["reduce_epi"], r["drain_sync"]]
        for i, v in enumerate(vals):
            tot[i] += v or 0.0
        cells = [name] + ["-" if v is None else f"{v:.2f}" for v in vals]
        print(("| " + " | ".join(cells) + " |") if md else "  ".join(f"{c:>10}" for c in cells))
    cells = ["step"] + [f"{v:.2f}" for v in tot]
    print(("| " + " | ".join(cells) + " |") if md else "  ".join(f"{c:>10}" for c in cells))
    print(f"(sampled step {d['sampled_step_us'][0]} us, {d['ms_per_batch']} ms per batch; rANS: its work "
          f"{d['work_us_team0'][4]} us is the coder; clock from each op's cycles / work us)")


if __name__ == "__main__":
    main()
