#!/bin/bash
# round 3, GPU call 26: the sparse rANS speculation with one renormalisation test per four centre symbols (shipped
# library) -- rANS / team / parity GPU tests, then decode alone (team_exp) and the driver's bench command for the
# previous library (liblbic_prev.so), the shipped one, and the LDS-staged split-GEMM slice (liblbic_wpre.so,
# LBIC_TEAM_WPRE=1, on top of the shipped one).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_rans_gpu.py tests/test_team_gpu.py tests/test_team_reference_gpu.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r03_c26_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r03_c26_tests.log; exit 3; }
tail -2 $O/r03_c26_tests.log
LBIC_LIB_VARIANT=wpre LBIC_TEAM_WPRE=1 timeout -k 10 300 python3 -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r03_c26_tests_wpre.log 2>&1 || { echo "wpre tests failed"; tail -30 $O/r03_c26_tests_wpre.log; exit 3; }
tail -2 $O/r03_c26_tests_wpre.log
te() {  # tag, env...
  local tag=$1; shift
  env "$@" TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r03_c26te_$tag.log 2>&1 || { echo "team_exp $tag failed"; tail -5 $O/r03_c26te_$tag.log; return 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean'], j['rans_done_us'][:6], j['gemm_beside_rans_done_us'][:6]) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r03_c26te_$tag.log $tag
}
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_c26_$tag.txt 2> $O/r03_c26_$tag.log || { echo "bench $tag failed"; tail -5 $O/r03_c26_$tag.log; return 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_c26_$tag.txt $tag
}
te prev LBIC_LIB_VARIANT=prev && te new LBIC_TEAM_WPRE=0 && te wpre LBIC_LIB_VARIANT=wpre LBIC_TEAM_WPRE=1 && \
run prev LBIC_LIB_VARIANT=prev && run new LBIC_TEAM_WPRE=0 && run wpre LBIC_LIB_VARIANT=wpre LBIC_TEAM_WPRE=1
