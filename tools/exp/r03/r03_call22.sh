#!/bin/bash
# round 3, GPU call 22: team GPU tests (incl. row-tile groups and the LDS table copy), then decode alone
# (tools/team_exp.py, 8 x 32 x 768^2 in one launch) and the driver's bench command for the four combinations of
# LBIC_TEAM_GROUPS (one barrier per 16-image row tile) and LBIC_TEAM_SPARSE_LDS (far rANS symbols from LDS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r03_c22_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r03_c22_tests.log; exit 3; }
tail -2 $O/r03_c22_tests.log
for v in 00 01 10 11; do
  g=${v:0:1}; l=${v:1:1}
  LBIC_TEAM_GROUPS=$g LBIC_TEAM_SPARSE_LDS=$l TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r03_grp_$v.log 2>&1 || { echo "team_exp $v failed"; tail -5 $O/r03_grp_$v.log; exit 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean'], j['rans_done_us'][:16], j['gemm_beside_rans_done_us'][:8]) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r03_grp_$v.log $v
done
for v in 00 01 10 11; do
  g=${v:0:1}; l=${v:1:1}
  LBIC_TEAM_GROUPS=$g LBIC_TEAM_SPARSE_LDS=$l timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_benchgrp_$v.txt 2> $O/r03_benchgrp_$v.log || { echo "bench $v failed"; tail -5 $O/r03_benchgrp_$v.log; exit 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_benchgrp_$v.txt $v
done
