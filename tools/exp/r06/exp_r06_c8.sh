#!/bin/bash
# r06 call 8: next-operation weight prefetch into LDS: timing on/off (same box), diag stamps, team + reference tests
set -eo pipefail
mkdir -p gpurun_out/r06
export SKIP_GRAPH=1 TEAMS=16 LBIC_TEAM_VERBOSE=1
for rep in 1 2; do
  for pf in 1 0; do
    echo "== pf $pf rep $rep" >> gpurun_out/r06/c8_ab.log
    PF=$pf timeout -k 10 200 python -u tools/team_exp.py 2>&1 | grep -E "decoder|team decode" >> gpurun_out/r06/c8_ab.log
  done
done
LBIC_LIB_VARIANT=tdiag RAW_OUT=gpurun_out/r06/c8_raw timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c8_te16_diag.log 2>&1
unset SKIP_GRAPH TEAMS LBIC_TEAM_VERBOSE
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_team_gpu.py tests/test_team_reference_gpu.py tests/test_one_gpu.py > gpurun_out/r06/c8_tests.log 2>&1
echo done
