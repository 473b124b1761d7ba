#!/bin/bash
# round 5, GPU call 31: the split GEMM's second phase dealt over all eight waves (team_gemm_tail; LBIC_TEAM_TAIL=0 turns it off)
# -- team tests; team decode alone 16 x 32 on / off; bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c31_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c31_tests.log; exit 3; }
tail -1 $O/r05_c31_tests.log
for c in 1 0; do
  LBIC_TEAM_TAIL=$c TEAMS=16 BATCH=32 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c31_te_c$c.log 2>&1 || { echo "team_exp $c failed"; tail -5 $O/r05_c31_te_c$c.log; exit 5; }
  python3 -c "import json,sys; [print('team tail', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c31_te_c$c.log $c
done
for c in 1 0 1 0; do
  LBIC_TEAM_TAIL=$c timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r05_c31_bench_c$c.log 2>&1 || { echo "bench $c failed"; tail -5 $O/r05_c31_bench_c$c.log; exit 6; }
  grep '^{' $O/r05_c31_bench_c$c.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench tail', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], j['quality']['enc_dec_bit_exact'])" $c
done
