#!/bin/bash
# round 3, GPU call 20: team GEMM prefetch depth.  Decode alone (tools/team_exp.py, 8 batches of 32 x 768^2 in one
# k_dec_team launch) and the driver's bench command for: the shipped library (next item prefetched for slices of <= 7
# k-blocks, 128-VGPR cap), liblbic_pf.so (next item at every slice length, 168-VGPR cap) and liblbic_deep.so (two
# items ahead, 256-VGPR cap).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for v in base pf deep; do
  if [ $v = base ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
  TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r03_teamdeep_$v.log 2>&1 || { echo "team_exp $v failed"; tail -5 $O/r03_teamdeep_$v.log; exit 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r03_teamdeep_$v.log $v
done
for v in base pf deep; do
  if [ $v = base ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
  timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_benchdeep_$v.txt 2> $O/r03_benchdeep_$v.log || { echo "bench $v failed"; tail -5 $O/r03_benchdeep_$v.log; exit 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_benchdeep_$v.txt $v
done
