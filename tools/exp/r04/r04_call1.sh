#!/bin/bash
# round 4, GPU call 1: the parked one-check rANS speculation measured once as a variant library
# (liblbic_onecheck.so, -DLBIC_RANS_ONE_CHECK) beside the shipped build: GPU rANS / team / team-vs-reference tests under
# the variant, decode alone (tools/team_exp.py, 8 teams) and the driver's bench command for both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
LBIC_LIB_VARIANT=onecheck timeout -k 10 400 python3 -u -m pytest tests/test_rans_gpu.py tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r04_c1_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r04_c1_tests.log; exit 3; }
tail -1 $O/r04_c1_tests.log
te() {  # tag, env...
  local tag=$1; shift
  env "$@" TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r04_c1te_$tag.log 2>&1 || { echo "team_exp $tag failed"; tail -5 $O/r04_c1te_$tag.log; return 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean'], j['rans_done_us'][:4]) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r04_c1te_$tag.log $tag
}
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r04_c1_$tag.txt 2> $O/r04_c1_$tag.log || { echo "bench $tag failed"; tail -5 $O/r04_c1_$tag.log; return 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r04_c1_$tag.txt $tag
}
te shipped && te onecheck LBIC_LIB_VARIANT=onecheck && te shipped2 && te onecheck2 LBIC_LIB_VARIANT=onecheck && \
run shipped && run onecheck LBIC_LIB_VARIANT=onecheck
