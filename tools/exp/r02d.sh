set -eo pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
B=$R/learned-block-based-image-compression_amd/csrc/build
for v in 0 1; do timeout -k 5 60 $B/rans_bench_stamps 32 96 0 63 $v 0.05; timeout -k 5 60 $B/rans_bench_stamps 32 96 0 30 $v 0.05; done > $O/rans_stamps_r02d.log 2>&1
timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 > $O/bench_r02d_base.log 2>&1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 > $O/bench_r02d_devkarg.log 2>&1
echo ok
