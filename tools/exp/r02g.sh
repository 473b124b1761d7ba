set -eo pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/gpu_tests_r02g.log 2>&1
LBIC_LIB_VARIANT=diag timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 > $O/diag_r02g.log 2>&1
timeout -k 10 400 python3 -u bench.py --cpu-budget 0 > $O/bench_r02g.log 2>&1
echo ok
