#!/bin/bash
# round 4, GPU call 6: the encoder's forked graph kept under sampling, stamps of EVERY encoder replay averaged
# (k_gemm launch duration of the bench line): the driver's bench command with and without the encoder stamps, then
# the same command under rocprofv3 (line vs trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --enc-sample-every 0 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r04_c6_nostamp.log 2>&1 || { echo "bench nostamp failed"; tail -20 $O/r04_c6_nostamp.log; exit 3; }
grep '^{' $O/r04_c6_nostamp.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('nostamp', j['value'], j['ms_per_step'], j['phases_ms_per_step'], json.dumps(j['kernels']['k_gemm']))"
bash tools/gpu_round.sh r04c6 notests --steps 20 --warmup 5 || { echo "gpu_round failed"; exit 5; }
grep '^{' $O/bench_r04c6.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact']); print(json.dumps(j['roofline']['per_kernel'])); print(json.dumps(j['kernels']['k_gemm']))"
grep '^{' $O/bench_rocprof_r04c6.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('traced run', j['value'], json.dumps(j['kernels']['k_gemm']))"
cat $O/kernel_stats_r04c6.txt
