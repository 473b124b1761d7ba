#!/bin/bash
# round 5, GPU call 23: the first decode launch's footprint beside the encoder (4 batches): 4 teams of 32 workgroups
# over 8 XCDs (default), of 16 per XCD over 8 XCDs (--first-team-size 16: half of every XCD's CUs), of 16 over 4 XCDs
# (+ LBIC_TEAM_SPREAD=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in def h16 q16 def h16 q16; do
  unset LBIC_TEAM_SPREAD; X=""
  if [ $v = h16 ]; then X="--first-team-size 16"; fi
  if [ $v = q16 ]; then X="--first-team-size 16"; export LBIC_TEAM_SPREAD=1; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 $X > $O/r05_c23_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c23_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c23_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], k['modes'])" $v
done
