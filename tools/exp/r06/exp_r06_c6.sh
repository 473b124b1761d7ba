#!/bin/bash
# r06 call 6: adopted team kernel (small code, selects kept): timing x2, diag stamps, team/reference tests
set -eo pipefail
mkdir -p gpurun_out/r06
export SKIP_GRAPH=1 TEAMS=16
timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c6_te16.log 2>&1
LBIC_LIB_VARIANT=tdiag RAW_OUT=gpurun_out/r06/c6_raw timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c6_te16_diag.log 2>&1
timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c6_te16b.log 2>&1
unset SKIP_GRAPH TEAMS
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_team_gpu.py tests/test_team_reference_gpu.py tests/test_one_gpu.py > gpurun_out/r06/c6_tests.log 2>&1
echo done
