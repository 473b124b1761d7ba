#!/bin/bash
# round 5, GPU call 12: 64 images per team (fast path to 10 tiles per workgroup, two rANS waves, the coder not inlined)
# -- the team tests; team decode alone at 32 and 64 images per team against HEAD (liblbic_prev.so); the driver's bench
# with two batches per team (new default) and with one.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c12_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c12_tests.log; exit 3; }
tail -1 $O/r05_c12_tests.log
for cfg in "32 8 main" "64 8 main" "32 8 prev" "64 4 main"; do
  set -- $cfg
  unset LBIC_LIB_VARIANT
  if [ $3 = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  TEAMS=$2 BATCH=$1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c12_te_b$1_t$2_$3.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c12_te_b$1_t$2_$3.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c12_te_b$1_t$2_$3.log "$cfg"
done
unset LBIC_LIB_VARIANT
for tb in 2 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --team-batches $tb > $O/r05_c12_bench_tb$tb.log 2>&1 || { echo "bench $tb failed"; tail -5 $O/r05_c12_bench_tb$tb.log; exit 6; }
  grep '^{' $O/r05_c12_bench_tb$tb.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', sys.argv[1], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_dec_team']['launch_ms_per_batch'], j['quality']['enc_dec_bit_exact'], j['roofline']['kernel'], j['roofline']['bound'], j['roofline']['frac'])" $tb
done
