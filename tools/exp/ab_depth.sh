set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for d in ${DEPTHS:-2 3 4}; do
  timeout -k 10 400 python3 bench.py --depth $d --steps ${STEPS:-12} --cpu-budget 0 --substream-steps 0 --serial-steps 0 > gpurun_out/depth_$d.log 2>&1 || exit 1
  echo "depth=$d $(tail -1 gpurun_out/depth_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms_per_step'])")"
done
