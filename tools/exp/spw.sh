set -eo pipefail
O=gpurun_out; mkdir -p $O
LBIC_SMALL_SPW=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/spw_tests.log 2>&1
tail -1 $O/spw_tests.log
for v in 2 1 2 1; do
  LBIC_SMALL_SPW=$v timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 2 > $O/spw_$v.log 2>&1
  grep '^{' $O/spw_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('spw $v', d['value'], d['ms_per_step'], d['phases_ms_per_step'], 'serial', d['serial_schedule']['phases_ms_per_step'], {n: (v['avg_span_us'], v['avg_launch_us']) for n, v in k.items()})"
done
