set -eo pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
LBIC_LIB_VARIANT=diag timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 > $O/diag_w4.log 2>&1
LBIC_LIB_VARIANT=diag timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 --workers 0 --depth 1 --steps 4 --warmup 1 > $O/diag_d1.log 2>&1
grep "diag k_gemm_s" $O/diag_w4.log | tail -1; grep "diag k_gemm_s" $O/diag_d1.log | tail -1
