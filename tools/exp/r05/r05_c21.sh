#!/bin/bash
# round 5, GPU call 21: teams of 16 workgroups decoding one 32-frame batch (9 tiles per workgroup, two rANS waves: the
# per-workgroup work of a 64-image team of 32) -- is a 16-workgroup team's raster step as fast as a 32-workgroup
# team's at twice the images?  8 teams alone (half the CUs busy), against 8 x 32 x 64 and 8 x 32 x 32.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for cfg in "32 8 16" "64 8 0" "32 8 0" "32 4 16"; do
  set -- $cfg
  TEAMS=$2 BATCH=$1 TEAM_SIZE=$3 LBIC_TEAM_SPREAD=1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c21_te_b$1_t$2_s$3.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c21_te_b$1_t$2_s$3.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c21_te_b$1_t$2_s$3.log "$cfg"
done
