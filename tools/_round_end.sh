#!/bin/bash
# GPU tests, the default bench line, then rocprofv3 kernel-trace stats of the bench's timed pipeline
# at --gang 16 (the default gang-32 command crashes inside rocprofv3 7.2's tracer).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python3 $R/bench.py > $O/bench.log 2>&1
cd /tmp && rm -rf /tmp/pk16
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk16 -o run -- \
    python3 $R/bench.py --cpu-budget 0 --substream-steps 0 --serial-steps 0 --gang 16 > $O/prof_kt16.log 2>&1
cp $(find /tmp/pk16 -name "*kernel_stats.csv") $O/kernel_stats_g16.csv
echo done
