#!/bin/bash
# round 5, GPU call 16: the first decode launch (4 batches beside the encoder) in three geometries -- 2 teams of 64
# images over 4 XCDs (default), LBIC_TEAM_SPREAD=4 (2 teams of 64 over all 8 XCDs), --first-team-batches 1 (4 teams of
# 32 over all 8 XCDs) -- and launch sizes 6,14.  The encoder's launches finish with their slowest XCD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in def sp4 ftb1 s614 def sp4 ftb1 s614; do
  unset LBIC_TEAM_SPREAD; X=""
  if [ $v = sp4 ]; then export LBIC_TEAM_SPREAD=4; fi
  if [ $v = ftb1 ]; then X="--first-team-batches 1"; fi
  if [ $v = s614 ]; then X="--team-sizes 6,14"; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 $X > $O/r05_c16_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c16_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c16_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'])" $v
done
