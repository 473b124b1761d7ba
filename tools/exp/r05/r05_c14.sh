#!/bin/bash
# round 5, GPU call 14: the team rANS call with its inputs from the kernarg segment (scalar) and an LDS pointer;
# bench (default schedule) twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_team_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c14_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c14_tests.log; exit 3; }
tail -1 $O/r05_c14_tests.log
for cfg in "32 8 main" "64 8 main" "32 8 prev"; do
  set -- $cfg
  unset LBIC_LIB_VARIANT
  if [ $3 = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  TEAMS=$2 BATCH=$1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c14_te_b$1_t$2_$3.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c14_te_b$1_t$2_$3.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c14_te_b$1_t$2_$3.log "$cfg"
done
unset LBIC_LIB_VARIANT
for v in def def; do
  unset LBIC_TEAM_SPREAD; X=""
  if [ $v = sp1 ]; then export LBIC_TEAM_SPREAD=1; fi
  if [ $v = s812 ]; then X="--team-sizes 8,12"; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 $X > $O/r05_c14_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c14_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c14_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', sys.argv[1], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_dec_team']['launch_ms_per_batch'], j['kernels']['k_dec_team']['avg_launch_us'], j['quality']['enc_dec_bit_exact'], j['roofline']['frac'])" $v
done
