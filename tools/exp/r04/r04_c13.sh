#!/bin/bash
# round 4, GPU call 13: the headline A/B on one box -- HEAD vs the call-11 tree (liblbic_c11.so: before the chain-select
# removal), the driver's command without the side legs, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r04_c13_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 $O/r04_c13_$tag.log; return 3; }
  grep '^{' $O/r04_c13_$tag.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(sys.argv[1], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_gemm']['avg_launch_us'], j['kernels']['k_dec_team']['launch_ms_per_batch'])" $tag
}
run head1 && run c11a LBIC_LIB_VARIANT=c11 && run head2 && run c11b LBIC_LIB_VARIANT=c11
