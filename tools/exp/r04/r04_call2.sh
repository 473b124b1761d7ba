#!/bin/bash
# round 4, GPU call 2: the tree after removing the rejected options and shipping the one-check rANS:
# the whole GPU suite, then the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/r04_c2_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r04_c2_tests.log; exit 3; }
tail -1 $O/r04_c2_tests.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/r04_c2_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r04_c2_bench.log; exit 4; }
grep '^{' $O/r04_c2_bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'), j['per_image'])"
