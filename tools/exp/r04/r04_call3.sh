#!/bin/bash
# round 4, GPU call 3: the weight-ring team decoder (loader waves + LDS-DMA rings) -- team GPU tests with the ring on and
# off, decode alone (team_exp.py, 8 teams) ring on vs off, then the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_team_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread -k "equals_graph" > $O/r04_c3_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c3_tests.log; exit 3; }
tail -1 $O/r04_c3_tests.log
te() {  # tag, env...
  local tag=$1; shift
  env "$@" TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r04_c3te_$tag.log 2>&1 || { echo "team_exp $tag failed"; tail -5 $O/r04_c3te_$tag.log; return 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][:2], j['op_us_mean'], j['rans_done_us'][:2]) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r04_c3te_$tag.log $tag
}
te ring LBIC_TEAM_RING=1 && te noring LBIC_TEAM_RING=0 || exit 4
timeout -k 10 700 python -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r04_c3_tests2.log 2>&1 || { echo "tests2 failed"; tail -40 $O/r04_c3_tests2.log; exit 5; }
tail -1 $O/r04_c3_tests2.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r04_c3_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r04_c3_bench.log; exit 6; }
grep '^{' $O/r04_c3_bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))"
