#!/bin/bash
# r06 call 13: team prologue quotients (cur vs thead), encoder single-segment k_gemm (cur vs khead), parity tests
set -eo pipefail
mkdir -p gpurun_out/r06
bash tools/exp/r06/exp_r06_ab.sh gpurun_out/r06/c13_ab.log 2 thead cur
for rep in 1 2; do
  for v in khead cur; do
    if [ $v = cur ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
    echo "== $v rep $rep" >> gpurun_out/r06/c13_enc.log
    timeout -k 10 120 python -u tools/enc_exp.py 2>&1 | grep encode_ms >> gpurun_out/r06/c13_enc.log
  done
done
unset LBIC_LIB_VARIANT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_fullsize_gpu.py tests/test_team_gpu.py tests/test_threads_gpu.py > gpurun_out/r06/c13_tests.log 2>&1
echo done
