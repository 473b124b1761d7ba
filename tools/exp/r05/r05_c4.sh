#!/bin/bash
# round 5, GPU call 4: k_gemm_t v4 (one group, software-pipelined LDS reads) ring depths 4/5/6 against k_gemm -- encoder alone,
# digests must match; then the whole GPU suite and the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for t in 0 4 5 6 4; do
  LBIC_ENC_TILED=$t timeout -k 10 240 python3 -u tools/enc_exp.py >> $O/r05_c4_enc.log 2>&1 || { echo "enc_exp failed"; tail -20 $O/r05_c4_enc.log; exit 2; }
done
grep encode_ms $O/r05_c4_enc.log
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c4_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c4_tests.log; exit 3; }
tail -1 $O/r05_c4_tests.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/r05_c4_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r05_c4_bench.log; exit 4; }
tail -1 $O/r05_c4_bench.log | cut -c1-400
# per-shape launch times of one encode, both kernels (rocprofv3 kernel trace)
cd /tmp && export TMPDIR=/tmp
for t in 0 4; do
  rm -rf /tmp/es$t
  LBIC_ENC_TILED=$t timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/es$t -o run -- python3 $R/tools/enc_exp.py > $O/r05_c4_es$t.log 2>&1 || { echo "rocprof $t failed"; exit 5; }
  python3 $R/tools/enc_shapes.py $(find /tmp/es$t -name "*kernel_trace.csv" | head -1) > $O/r05_c4_shapes$t.txt
  head -25 $O/r05_c4_shapes$t.txt
done
