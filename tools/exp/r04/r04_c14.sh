#!/bin/bash
# round 4, GPU call 14: k_dec_one phase stamps (the workgroup holding column tile 0 of each op: inputs there, registers
# loaded, chain done, reduced, published, shader clock) and the gran1 fast path: single-image tests + timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/r04_c14_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c14_tests.log; exit 3; }
tail -1 $O/r04_c14_tests.log
timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c14_one.log 2>&1 || { echo "one_exp failed"; tail -10 $O/r04_c14_one.log; exit 4; }
grep '^{' $O/r04_c14_one.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r04_c14_bench.log 2>&1 || { echo "bench failed"; tail -5 $O/r04_c14_bench.log; exit 5; }
grep '^{' $O/r04_c14_bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_gemm']['avg_launch_us'], j['kernels']['k_dec_team']['launch_ms_per_batch'])"
