"""Aggregate rocprofv3 --pmc CSV output into per-kernel averages (per dispatch).

usage: python tools/pmc_summary.py OUT.json DIR [DIR ...]
Each DIR is a rocprofv3 -d output directory of one --pmc pass (FETCH_SIZE and WRITE_SIZE need separate
passes on gfx950: MI355X_MICROARCH.md "rocprofv3 PMC slots").  Writes {kernel: {counter: mean, "dispatches": n}}
and, per kernel, "hbm_bytes_per_dispatch" = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH_SIZE counts half of
the bytes of a wide coalesced read on gfx950: MI355X_MICROARCH.md "HBM").
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(lbic::\w+\)$", "", name)
    return name.replace("lbic::", "").replace(" ", "")


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    # kernel families (template arguments dropped), dispatch-weighted
    fam = defaultdict(lambda: defaultdict(list))
    for k, cs in list(acc.items()):
        f = re.sub(r"<.*>$", "", k)
        if f != k:
            for c, v in cs.items():
                fam[f][c].extend(v)
    acc.update(fam)
    res = {}
    for k, cs in acc.items():
        r = {c: sum(v) / len(v) for c, v in cs.items()}
        r["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            r["hbm_bytes_per_dispatch"] = (2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024
        res[k] = r
    res["_source"] = {"dirs": dirs, "note": "per-dispatch means over every dispatch of the profiled command"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, r in sorted(res.items()):
        if not k.startswith("_"):
            print(k, {c: round(v, 1) for c, v in r.items()})


if __name__ == "__main__":
    main()
