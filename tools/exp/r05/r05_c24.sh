#!/bin/bash
# round 5, GPU call 24: the first launch's team size per XCD slot (8 / 12 / 16 / 20) and the group split (4+16, 6+14,
# 8+12) with half-XCD teams in the first launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in h16 h8 h12 h20 s614 s812 h16 h8 h12 h20 s614 s812; do
  X=""
  case $v in
    h8) X="--first-team-size 8";; h12) X="--first-team-size 12";; h20) X="--first-team-size 20";;
    s614) X="--team-sizes 6,14";; s812) X="--team-sizes 8,12";;
  esac
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 $X > $O/r05_c24_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c24_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c24_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'])" $v
done
