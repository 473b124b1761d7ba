#!/bin/bash
# One GPU session: GPU tests, the driver's bench command, then rocprofv3 kernel-trace stats of the SAME
# command (the roofline's avg launch duration must agree with that summary).  Outputs under gpurun_out/.
# usage: tools/gpu_round.sh TAG [tests|notests] [extra bench args...]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-x}
MODE=${2:-tests}
shift 2 || true
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "$MODE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
fi
timeout -k 10 500 python3 -u $R/bench.py --gpus 1 "$@" > $O/bench_$TAG.log 2>&1
cd /tmp && rm -rf /tmp/pk_$TAG
rc=0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk_$TAG -o run -- \
    python3 $R/bench.py --gpus 1 "$@" > $O/bench_rocprof_$TAG.log 2>&1 || rc=$?
# (no further GPU step after a failure; the summaries are copied either way)
cp $(find /tmp/pk_$TAG -name "*kernel_stats.csv") $O/kernel_stats_$TAG.csv || true
python3 $R/tools/kstats_summary.py $O/kernel_stats_$TAG.csv $(find /tmp/pk_$TAG -name "*kernel_trace.csv" | head -1) \
    > $O/kernel_stats_$TAG.txt || true
echo "done rc=$rc"
exit $rc
