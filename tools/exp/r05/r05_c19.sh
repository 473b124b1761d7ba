#!/bin/bash
# round 5, GPU call 19: the team tests (new: the sparse coder at > 1 bit per symbol with two rANS waves); configs 4 and
# 3 (all 24 frames) with one and two batches per team (the dense tables may not fit beside a 64-image geometry's
# partials: lbc_decode_team now switches to the sparse coder instead of the row graphs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_team_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c19_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c19_tests.log; exit 3; }
tail -1 $O/r05_c19_tests.log
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
run() {  # name, timeout, args...
  local f=$1 t=$2; shift 2
  timeout -k 10 $t $B "$@" > $O/${f}.log 2>&1 || { echo "$f failed"; tail -5 $O/${f}.log; return 3; }
  grep '^{' $O/${f}.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels'].get('k_dec_team',{})
print('$f', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['bpp'], d['quality']['enc_dec_bit_exact'], k.get('launch_windows_s'), k.get('avg_launch_us'))"
}
run r05_c19_cfg4_tb2 500 --config B4_highrate --size 768 --batch 32 --steps 6 --warmup 3 --team-batches 2 && \
run r05_c19_cfg4_tb1 400 --config B4_highrate --size 768 --batch 32 --steps 6 --warmup 3 --team-batches 1 && \
run r05_c19_cfg3_all24_tb1 400 --config B8_highrate --size 768 --height 512 --batch 24 --steps 8 --warmup 3 --team-batches 1
