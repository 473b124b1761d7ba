set -eo pipefail
O=gpurun_out; mkdir -p $O
LBIC_DEC_ROWS_PER_GRAPH=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/rpg_tests.log 2>&1
tail -1 $O/rpg_tests.log
for r in 1 4 12 2 8 1; do
  LBIC_DEC_ROWS_PER_GRAPH=$r timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 2 > $O/rpg_$r.log 2>&1
  grep '^{' $O/rpg_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rpg $r', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], 'serial', d['serial_schedule']['phases_ms_per_step'])"
done
