#!/bin/bash
# round 5, GPU call 9: the encoder's XCD rectangles (k_gemm, LBIC_ENC_XPART=1: each XCD fetches 1/RG of the A rows and
# 1/CG of the weights) -- measured alone in round 3 (6 % slower), never beside the team decoder: encoder alone (digest
# must match), the GPU tests that encode, then the driver's bench alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for x in 0 1 0 1; do
  LBIC_ENC_XPART=$x timeout -k 10 240 python3 -u tools/enc_exp.py > $O/r05_c9_enc_x$x.log 2>&1 || { echo "enc_exp failed"; tail -5 $O/r05_c9_enc_x$x.log; exit 2; }
  echo "x$x $(grep encode_ms $O/r05_c9_enc_x$x.log)"
done
LBIC_ENC_XPART=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c9_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r05_c9_tests.log; exit 3; }
tail -1 $O/r05_c9_tests.log
for x in 1 0 1 0; do
  LBIC_ENC_XPART=$x timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r05_c9_bench_x$x.log 2>&1 || { echo "bench $x failed"; tail -5 $O/r05_c9_bench_x$x.log; exit 6; }
  grep '^{' $O/r05_c9_bench_x$x.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', sys.argv[1], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_dec_team']['launch_ms_per_batch'], j['roofline']['per_kernel']['k_gemm']['avg_launch_us'])" x$x
done
