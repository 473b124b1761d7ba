#!/bin/bash
# round 3, GPU call 14: which hardware queues the encoder's and the team decoder's streams land on
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
run() {  # tag pre gap hwq
  LBIC_BENCH_STREAM_PRE=$2 LBIC_BENCH_STREAM_GAP=$3 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --hw-queues $4 > $O/r03_q_$1.log 2>&1 || exit 2
  grep '^{' $O/r03_q_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 pre=$2 gap=$3 hwq=$4', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
}
run a 0 0 8
run b 0 1 8
run c 1 0 8
run d 0 2 8
run e 0 3 8
run f 0 0 4
run g 0 0 16
run h 2 0 8
