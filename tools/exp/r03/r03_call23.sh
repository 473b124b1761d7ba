#!/bin/bash
# round 3, GPU call 23: beside the encoder, the driver's bench command with the team decoder's waves at a higher issue
# priority (LBIC_TEAM_PRIO = s_setprio level; 0 = default), and the encoder tile shapes 32x32 / 8 waves (LBIC_ENC_CFG 13)
# and 16x64 / 8 (12) -- measured alone only in rounds 2-3.  Extra env for every run: $EXTRA (e.g. the best call-22 mode).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_c23_$tag.txt 2> $O/r03_c23_$tag.log || { echo "bench $tag failed"; tail -5 $O/r03_c23_$tag.log; return 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_c23_$tag.txt $tag
}
run prio0 LBIC_TEAM_PRIO=0 $EXTRA && run prio3 LBIC_TEAM_PRIO=3 $EXTRA && run prio1 LBIC_TEAM_PRIO=1 $EXTRA && \
run enc13 LBIC_ENC_CFG=13 $EXTRA && run enc12 LBIC_ENC_CFG=12 $EXTRA
