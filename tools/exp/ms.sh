set -eo pipefail
O=gpurun_out; mkdir -p $O
LBIC_SMALL_MS=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/ms2_tests.log 2>&1
tail -1 $O/ms2_tests.log
for ms in 2 1 2 1; do
  LBIC_SMALL_MS=$ms timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 2 > $O/ms_$ms.log 2>&1
  grep '^{' $O/ms_$ms.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms $ms', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['avg_span_us'], 'serial', d['serial_schedule']['phases_ms_per_step'])"
done
