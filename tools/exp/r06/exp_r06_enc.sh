#!/bin/bash
# r06: encoder launch accounting: rocprofv3 kernel trace of one 32-frame 768x768 B8_lowrate
# compress (tools/enc_exp.py, REPS=1) -> tools/enc_rounds.py
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && rm -rf /tmp/enc_kt
REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/enc_kt -o run -- python3 $R/tools/enc_exp.py > $O/enc_trace.log 2>&1
python3 $R/tools/enc_rounds.py /tmp/enc_kt > $O/enc_rounds.json
echo enc done
