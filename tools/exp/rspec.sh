set -eo pipefail
O=gpurun_out; mkdir -p $O
B=learned-block-based-image-compression_amd/csrc/build
timeout -k 10 300 python -u -m pytest tests/test_rans_gpu.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/rspec_tests.log 2>&1
tail -1 $O/rspec_tests.log
for sp in 0.05 0.1 0.2 0.4; do timeout -k 5 60 $B/rans_bench_stamps 32 96 0 30 1 $sp; done > $O/rspec_stamps.log 2>&1
cat $O/rspec_stamps.log
for v in new prev new prev; do
  if [ $v = prev ]; then export LBIC_LIB_VARIANT=prev; else unset LBIC_LIB_VARIANT; fi
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 > $O/rspec_$v.log 2>&1
  grep '^{' $O/rspec_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v', d['value'], d['ms_per_step'], d['phases_ms_per_step'], {n: (v['avg_span_us'], v['avg_launch_us']) for n, v in k.items()})"
done
