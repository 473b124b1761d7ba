#!/bin/bash
# A/B of a liblbic environment toggle on the serial bench (encode / decode phases), two rounds each:
#   [ROUNDS=n] bash tools/ab_env.sh VAR "v1 v2"
set -o pipefail
VAR=$1; VALS=$2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -20 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
S="python3 bench.py --serial --steps 2 --cpu-budget 0 --substream-steps 0 --serial-steps 0"
for r in $(seq ${ROUNDS:-2}); do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 $S > gpurun_out/ab_${v}.log 2>&1 || exit 1
  echo "$VAR=$v $(tail -1 gpurun_out/ab_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})")"
done; done
