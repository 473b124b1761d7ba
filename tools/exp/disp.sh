set -eo pipefail
O=gpurun_out; mkdir -p $O
B=learned-block-based-image-compression_amd/csrc/build/dispatch_bench
export GPU_MAX_HW_QUEUES=8
( timeout -k 10 60 $B 96 0 2000 5 && timeout -k 10 60 $B 96 3000 1000 3 && timeout -k 10 60 $B 1 0 2000 5 && timeout -k 10 60 $B 256 0 2000 5 ) > $O/dispatch.txt 2>&1
cat $O/dispatch.txt
unset GPU_MAX_HW_QUEUES
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/fork_tests.log 2>&1
tail -1 $O/fork_tests.log
for f in 1 0; do
  LBIC_ENC_FORK=$f timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 2 > $O/fork_$f.log 2>&1
  grep '^{' $O/fork_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fork $f', d['value'], d['ms_per_step'], d['phases_ms_per_step'], 'serial', d['serial_schedule']['phases_ms_per_step'])"
done
