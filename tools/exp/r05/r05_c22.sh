#!/bin/bash
# round 5, GPU call 22: up to 16 teams per launch (two per XCD, each half its CUs) -- one 32-frame batch per team with
# the per-workgroup work of a 64-image team.  Team tests; team decode alone 16 x 32 vs 8 x 64; the bench's new default
# (--team 16) against the two-batch teams (--team 8 --team-batches 2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c22_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c22_tests.log; exit 3; }
tail -1 $O/r05_c22_tests.log
for cfg in "32 16" "64 8"; do
  set -- $cfg
  TEAMS=$2 BATCH=$1 SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c22_te_b$1_t$2.log 2>&1 || { echo "team_exp $cfg failed"; tail -5 $O/r05_c22_te_b$1_t$2.log; exit 5; }
  python3 -c "import json,sys; [print('team', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c22_te_b$1_t$2.log "$cfg"
done
for v in t16 t8b2 t16 t8b2; do
  X=""; if [ $v = t8b2 ]; then X="--team 8 --team-batches 2"; fi
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 $X > $O/r05_c22_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c22_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c22_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], k['modes'], j['quality']['enc_dec_bit_exact'])" $v
done
