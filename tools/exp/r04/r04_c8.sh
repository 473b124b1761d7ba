#!/bin/bash
# round 4, GPU call 8: k_dec_one with the bias prefetch, the GDN input from LDS, the left tap from d3's granules and lazy
# zpad drains: its GPU tests, the single-image decode timing + per-operation stamps (tools/one_exp.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py tests/test_fullsize_gpu.py -x -v -s -m gpu --timeout 180 --timeout-method thread > $O/r04_c8_one.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c8_one.log; exit 3; }
grep -E "path|passed|failed" $O/r04_c8_one.log | tail -8
timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c8_exp.log 2>&1 || { echo "one_exp failed"; tail -10 $O/r04_c8_exp.log; exit 4; }
cat $O/r04_c8_exp.log | grep '^{'
