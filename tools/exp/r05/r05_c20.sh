#!/bin/bash
# round 5, GPU call 20: next-item weight requests rolled into the chain for 8-9 k-block slices (k_dec_team) -- team
# tests; team decode alone at 64 and 32 images per team against the previous build (liblbic_prev.so); bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c20_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c20_tests.log; exit 3; }
tail -1 $O/r05_c20_tests.log
for cfg in "64 8 main" "64 8 prev" "32 8 main" "32 8 prev"; do
  set -- $cfg
  unset LBIC_LIB_VARIANT
  if [ $3 = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  TEAMS=$2 BATCH=$1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c20_te_b$1_t$2_$3.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c20_te_b$1_t$2_$3.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c20_te_b$1_t$2_$3.log "$cfg"
done
for v in main prev main prev; do
  unset LBIC_LIB_VARIANT
  if [ $v = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r05_c20_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c20_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c20_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], k['modes'])" $v
done
