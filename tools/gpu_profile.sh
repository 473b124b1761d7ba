#!/bin/bash
# One GPU session: the PMC passes (FETCH_SIZE, WRITE_SIZE separately) -- the decoder's kernels on a 128x128-frame
# run whose raster-step shapes equal the 768x768 config's (gang x 32 rows per step), the encoder's GEMMs on
# 768x768 encode-only passes -- merged into pmc_traffic.json, which the full bench line that follows reads for
# roofline.traffic; then rocprofv3 kernel-trace stats of the same bench command's timed pipeline (without the
# serial / two-stage / sub-stream side legs: with them, >1 M traced dispatches, rocprofv3 7.2 crashed once
# with SIGSEGV in its own thread after the warmup).  Outputs under gpurun_out/.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/pk /tmp/pf /tmp/pw /tmp/pef /tmp/pew
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 --size 128 --steps 4 --warmup 1 > $O/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 --size 128 --steps 4 --warmup 1 > $O/prof_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pef -o run -- \
    python3 $R/bench.py --encode-only 2 > $O/prof_enc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pew -o run -- \
    python3 $R/bench.py --encode-only 2 > $O/prof_enc_write.log 2>&1
python3 $R/tools/pmc_summary.py $O/pmc_small.json /tmp/pf /tmp/pw > $O/pmc_summary.txt
python3 $R/tools/pmc_summary.py $O/pmc_enc.json /tmp/pef /tmp/pew > $O/pmc_summary_enc768.txt
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
small, enc = json.load(open(o + "/pmc_small.json")), json.load(open(o + "/pmc_enc.json"))
for k, v in enc.items():        # encoder GEMMs from the 768x768 passes, the rest from the 128x128 run
    if k.startswith("k_gemm<") or k == "k_gemm":
        small[k] = dict(v, source="768x768 encode-only passes")
json.dump(small, open(o + "/pmc_traffic.json", "w"), indent=1)
PY
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json
timeout -k 10 400 python3 $R/bench.py > $O/bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 --serial-steps 0 > $O/prof_kt.log 2>&1
cp $(find /tmp/pk -name "*kernel_stats.csv") $O/kernel_stats.csv
echo done
