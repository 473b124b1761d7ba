#!/bin/bash
# round 5, GPU call 11: 64 images per team on the fast path (TEAM_NI_MAX 10, two rANS waves per workgroup) against
# HEAD's library (liblbic_prev.so): team decode alone, 32 and 64 images per team, per-operation stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for cfg in "32 8 main" "64 8 main" "32 8 prev" "64 8 prev" "64 4 main" "32 8 main"; do
  set -- $cfg
  unset LBIC_LIB_VARIANT
  if [ $3 = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  TEAMS=$2 BATCH=$1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c11_te_b$1_t$2_$3.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c11_te_b$1_t$2_$3.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean'], j['work_us_team0']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c11_te_b$1_t$2_$3.log "$cfg"
done
