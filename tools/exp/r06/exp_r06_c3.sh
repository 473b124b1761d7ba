#!/bin/bash
# r06 call 3: the team decoder after the code-size / chain-select changes: timing, stamps, tests, bench
set -eo pipefail
mkdir -p gpurun_out/r06
export SKIP_GRAPH=1
TEAMS=16 timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c3_te16.log 2>&1
LBIC_LIB_VARIANT=tdiag TEAMS=16 RAW_OUT=gpurun_out/r06/c3_raw timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c3_te16_diag.log 2>&1
unset SKIP_GRAPH
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_team_gpu.py tests/test_team_reference_gpu.py tests/test_gpu_parity.py tests/test_one_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r06/c3_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06/c3_bench.log 2>&1
echo done
