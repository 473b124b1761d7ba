#!/bin/bash
# round 5, GPU call 29: config 4 with two batches per team -- which path the launch took (kernels.k_dec_team.modes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
LBIC_TEAM_VERBOSE=1 timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0 --config B4_highrate --size 768 --batch 32 --steps 6 --warmup 3 --team-batches 2 > $O/r05_c29_cfg4_tb2.log 2>&1 || { echo "failed"; tail -5 $O/r05_c29_cfg4_tb2.log; exit 3; }
grep -v '^{' $O/r05_c29_cfg4_tb2.log | tail -5
grep '^{' $O/r05_c29_cfg4_tb2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']['k_dec_team']; print(d['value'], k['modes'], k['launch_windows_s'], k['avg_launch_us'], k['plain_handoffs'], k['barrier_timeout_fallbacks'])"
