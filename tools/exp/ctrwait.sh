set -eo pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/ctr_tests.log 2>&1
tail -1 $O/ctr_tests.log
for v in new prev new prev; do
  if [ $v = prev ]; then export LBIC_LIB_VARIANT=prev; else unset LBIC_LIB_VARIANT; fi
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 2 > $O/ctr_$v.log 2>&1
  grep '^{' $O/ctr_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v', d['value'], d['ms_per_step'], d['phases_ms_per_step'], 'serial', d['serial_schedule']['phases_ms_per_step'], {n: (v['avg_span_us'], v['avg_launch_us']) for n, v in k.items()})"
done
