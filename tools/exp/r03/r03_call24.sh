#!/bin/bash
# round 3, GPU call 24: the team decoder's persistent rANS coder state (LBIC_TEAM_RPERSIST, default 1): team GPU tests,
# decode alone (team_exp) and the driver's bench command with it off / on; then beside the encoder the team waves at
# issue priority 3 (LBIC_TEAM_PRIO) and the encoder's 32x32 / 8-wave tile (LBIC_ENC_CFG=13).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py tests/test_rans_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r03_c24_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r03_c24_tests.log; exit 3; }
tail -2 $O/r03_c24_tests.log
for v in 0 1; do
  LBIC_TEAM_RPERSIST=$v TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r03_rp_$v.log 2>&1 || { echo "team_exp $v failed"; tail -5 $O/r03_rp_$v.log; exit 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean'], j['rans_done_us'][:12], j['gemm_beside_rans_done_us'][:6]) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r03_rp_$v.log $v
done
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_c24_$tag.txt 2> $O/r03_c24_$tag.log || { echo "bench $tag failed"; tail -5 $O/r03_c24_$tag.log; return 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_c24_$tag.txt $tag
}
run rp0 LBIC_TEAM_RPERSIST=0 && run rp1 LBIC_TEAM_RPERSIST=1 && run prio3 LBIC_TEAM_PRIO=3 && run enc13 LBIC_ENC_CFG=13
