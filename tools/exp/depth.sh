set -eo pipefail
O=gpurun_out; mkdir -p $O
for d in 2 3 4 5 6; do
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 --depth $d > $O/depth_$d.log 2>&1
  grep '^{' $O/depth_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth', $d, d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['avg_span_us'])"
done
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 --depth 3 > $O/depth_3_q4.log 2>&1
grep '^{' $O/depth_3_q4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth 3 q4', d['value'], d['ms_per_step'], d['phases_ms_per_step'])"
