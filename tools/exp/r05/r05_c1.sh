#!/bin/bash
# round 5, GPU call 1: the LDS-staged encoder GEMM (k_gemm_t) against k_gemm -- encoder alone (digest must match),
# the GPU suite's encoder-heavy files, then the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for t in 0 1 0 1; do
  LBIC_ENC_TILED=$t timeout -k 10 240 python3 -u tools/enc_exp.py >> $O/r05_c1_enc.log 2>&1 || { echo "enc_exp failed"; tail -20 $O/r05_c1_enc.log; exit 2; }
done
cat $O/r05_c1_enc.log | grep encode_ms
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_team_gpu.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c1_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c1_tests.log; exit 3; }
tail -1 $O/r05_c1_tests.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/r05_c1_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05_c1_bench.log; exit 4; }
tail -1 $O/r05_c1_bench.log | cut -c1-600
