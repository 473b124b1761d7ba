set -eo pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_share.log 2>&1
tail -1 $O/gpu_tests_share.log
for sw in 1 0 1 0; do
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 --share-weights $sw > $O/share_$sw.log 2>&1
  grep '^{' $O/share_$sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('share $sw', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['avg_span_us'])"
done
