#!/bin/bash
# round 5, GPU call 2: k_gemm_t (slice loop, early-clobber reads) ring depths 4/6/8 against k_gemm -- encoder alone,
# digests must match; then the whole GPU suite and the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for t in 0 8 6 4 8; do
  LBIC_ENC_TILED=$t timeout -k 10 240 python3 -u tools/enc_exp.py >> $O/r05_c2_enc.log 2>&1 || { echo "enc_exp failed"; tail -20 $O/r05_c2_enc.log; exit 2; }
done
grep encode_ms $O/r05_c2_enc.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c2_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c2_tests.log; exit 3; }
tail -1 $O/r05_c2_tests.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/r05_c2_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05_c2_bench.log; exit 4; }
tail -1 $O/r05_c2_bench.log | cut -c1-400
