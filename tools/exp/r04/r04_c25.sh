#!/bin/bash
# round 4, GPU call 25: poll loops (k_dec_one waits, k_dec_team barriers) that read the clock only every 16th round
# (every round under a test's tiny timeout) -- liblbic_tmt.so -- against main: the whole GPU suite on tmt, then team
# decode alone, the driver's bench and single-image decode, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
LBIC_LIB_VARIANT=tmt timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/r04_c25_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c25_tests.log; exit 3; }
tail -1 $O/r04_c25_tests.log
for v in main tmt main tmt; do
  unset LBIC_LIB_VARIANT
  if [ $v = tmt ]; then export LBIC_LIB_VARIANT=tmt; fi
  TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u tools/team_exp.py > $O/r04_c25_te_$v.log 2>&1 || { echo "team_exp $v failed"; tail -5 $O/r04_c25_te_$v.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r04_c25_te_$v.log $v
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r04_c25_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r04_c25_bench_$v.log; exit 6; }
  grep '^{' $O/r04_c25_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', sys.argv[1], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_gemm']['avg_launch_us'], j['kernels']['k_dec_team']['launch_ms_per_batch'])" $v
  REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c25_one_$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c25_one_$v.log; exit 7; }
  echo "one $v"; grep '"decoder": "one"' $O/r04_c25_one_$v.log
done
