#!/bin/bash
# round 3, GPU call 19: CU-split team schedule (bench.py --dec-cus K: team decode launches on K CUs of every XCD, the
# encoder on the other 32 - K) against the shared default, driver command otherwise (--steps 20 --warmup 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for k in 0 16 12 20; do
  timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --dec-cus $k \
    > $O/r03_cusplit_$k.txt 2> $O/r03_cusplit_$k.log || { echo "dec-cus $k failed"; tail -5 $O/r03_cusplit_$k.log; exit 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('barrier_timeout_fallbacks'))" $O/r03_cusplit_$k.txt $k
done
