set -eo pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
B=$R/learned-block-based-image-compression_amd/csrc/build
for v in 0 1; do timeout -k 5 60 $B/rans_bench_stamps 32 96 0 63 $v 0.05; timeout -k 5 60 $B/rans_bench_stamps 32 96 0 30 $v 0.05; timeout -k 5 60 $B/rans_bench_stamps 32 96 0 30 $v 0.5; done > $O/rans_stamps_r02e.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_rans_gpu.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/gpu_tests_r02e.log 2>&1
bash tools/gpu_profile.sh
cp $O/pmc_traffic.json profiles/pmc_traffic.json
bash tools/gpu_round.sh r02e notests
