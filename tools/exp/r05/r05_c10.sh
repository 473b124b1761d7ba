#!/bin/bash
# round 5, GPU call 10: the team decoder with 64 images per team (two 32-frame batches as one, MT = 4 row tiles) against
# 32 per team -- per-operation stamps, to size a two-batch team schedule.  Current kernel: context layers 0-1 take the
# long path at 64 images (9 / 7.5 tiles per workgroup > TEAM_NI_MAX).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for cfg in "32 8" "64 8" "64 4" "32 8"; do
  set -- $cfg
  TEAMS=$2 BATCH=$1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c10_te_b$1_t$2.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c10_te_b$1_t$2.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean'], j['work_us_team0']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c10_te_b$1_t$2.log "$cfg"
done
