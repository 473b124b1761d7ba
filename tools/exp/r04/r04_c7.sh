#!/bin/bash
# round 4, GPU call 7: the single-image decoder k_dec_one (one.hip) -- its GPU tests first, then the whole suite; the
# driver's bench command (per-image decode through k_dec_one; encoder stamps over every replay) and the same command
# under rocprofv3; B16_lowrate's "low" point calibrated at the bench's 2048x2048 frames.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -s -m gpu --timeout 120 --timeout-method thread > $O/r04_c7_one.log 2>&1 || { echo "one tests failed"; tail -40 $O/r04_c7_one.log; exit 3; }
grep -E "path|passed|failed" $O/r04_c7_one.log | tail -12
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/r04_c7_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r04_c7_tests.log; exit 4; }
tail -1 $O/r04_c7_tests.log
bash tools/gpu_round.sh r04c7 notests --steps 20 --warmup 5 || { echo "gpu_round failed"; exit 5; }
grep '^{' $O/bench_r04c7.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact']); print(json.dumps(j['per_image'])); print(json.dumps(j['roofline']['per_kernel'])); print(json.dumps(j['kernels']['k_gemm']))"
grep '^{' $O/bench_rocprof_r04c7.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('traced run', j['value'], json.dumps(j['kernels']['k_gemm']))"
cat $O/kernel_stats_r04c7.txt
timeout -k 10 300 python3 -u tools/calib_low_gpu.py 0.120 2048 > $O/r04_c7_calib.log 2>&1 || { echo "calib failed"; tail -5 $O/r04_c7_calib.log; exit 6; }
tail -3 $O/r04_c7_calib.log
