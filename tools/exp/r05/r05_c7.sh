#!/bin/bash
# round 5, GPU call 7: context layer 0's row-above K slices one raster step early (k_dec_team, TeamArgs::pre_wy) --
# the team tests, then team decode alone (8 batches, per-operation stamps) and the driver's bench, alternated against
# HEAD's library (liblbic_prev.so) and LBIC_TEAM_PRE=0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c7_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c7_tests.log; exit 3; }
tail -1 $O/r05_c7_tests.log
for v in main prev nopre main prev; do
  unset LBIC_LIB_VARIANT LBIC_TEAM_PRE
  if [ $v = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  if [ $v = nopre ]; then export LBIC_TEAM_PRE=0; fi
  TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u tools/team_exp.py > $O/r05_c7_te_$v.log 2>&1 || { echo "team_exp $v failed"; tail -5 $O/r05_c7_te_$v.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c7_te_$v.log $v
done
for v in main prev main prev; do
  unset LBIC_LIB_VARIANT LBIC_TEAM_PRE
  if [ $v = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r05_c7_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c7_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c7_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', sys.argv[1], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_dec_team']['launch_ms_per_batch'])" $v
done
