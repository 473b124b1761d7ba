#!/bin/bash
# round 3, GPU call 7: encoder launch times by GEMM shape (rocprofv3 kernel trace of tools/enc_exp.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && rm -rf /tmp/et
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/et -o run -- python3 $R/tools/enc_exp.py > $O/r03_enc_trace.log 2>&1 || exit 3
python3 $R/tools/enc_shapes.py $(find /tmp/et -name "*kernel_trace.csv" | head -1) > $O/r03_enc_shapes.txt
head -3 $(find /tmp/et -name "*kernel_trace.csv" | head -1) > $O/r03_enc_trace_head.csv
cat $O/r03_enc_shapes.txt
