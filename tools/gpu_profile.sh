#!/bin/bash
# One GPU session: full bench line, rocprofv3 kernel-trace stats of the same command, and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) on a 128x128-frame run whose per-launch GEMM / rANS shapes equal the 768x768
# config's (M = 32 rows per step).  Outputs under gpurun_out/ (summaries only).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $O/bench.log 2>&1
cd /tmp
rm -rf /tmp/pk /tmp/pf /tmp/pw
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 > $O/prof_kt.log 2>&1
cp $(find /tmp/pk -name "*kernel_stats.csv") $O/kernel_stats.csv
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 --size 128 --steps 1 --warmup 1 > $O/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 --size 128 --steps 1 --warmup 1 > $O/prof_write.log 2>&1
python3 $R/tools/pmc_summary.py $O/pmc_traffic.json /tmp/pf /tmp/pw > $O/pmc_summary.txt
echo done
