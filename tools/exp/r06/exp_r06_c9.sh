#!/bin/bash
# r06 call 9: lean operation prologue (buffer-load addressing, one-segment instance): tests, A/B vs HEAD, diag stamps
set -eo pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_team_gpu.py tests/test_team_reference_gpu.py > gpurun_out/r06/c9_tests.log 2>&1
bash tools/exp/r06/exp_r06_ab.sh gpurun_out/r06/c9_ab.log 2 abhead cur
SKIP_GRAPH=1 TEAMS=16 LBIC_LIB_VARIANT=tdiag timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c9_te16_diag.log 2>&1
echo done
