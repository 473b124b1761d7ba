#!/bin/bash
# Encoder GEMM shape A/B: GPU parity tests under each LBIC_ENC_CFG value, then the serial bench (encode phase)
#   bash tools/ab_enc.sh "0 10 11"
set -o pipefail
mkdir -p gpurun_out
for v in $1; do
  LBIC_ENC_CFG=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/enc_tests_$v.log 2>&1 || { echo "cfg $v tests FAILED"; tail -30 gpurun_out/enc_tests_$v.log; exit 1; }
  echo "cfg $v: $(tail -1 gpurun_out/enc_tests_$v.log)"
done
S="python3 bench.py --serial --steps 2 --cpu-budget 0 --substream-steps 0 --serial-steps 0"
for r in 1 2; do for v in $1; do
  LBIC_ENC_CFG=$v timeout -k 10 300 $S > gpurun_out/enc_$v.log 2>&1 || exit 1
  echo "LBIC_ENC_CFG=$v $(tail -1 gpurun_out/enc_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})")"
done; done
