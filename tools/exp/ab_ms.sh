#!/bin/bash
# k_gemm_s row subtiles in ganged decoder raster steps: GPU parity tests under LBIC_DEC_MS=2 and 4, then the
# pipelined bench (gang 8, depth 2) for each value, two rounds
#   bash tools/ab_ms.sh "1 2 4"
set -o pipefail
mkdir -p gpurun_out
for v in 2 4; do
  LBIC_DEC_MS=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/ms_tests_$v.log 2>&1 || { echo "MS=$v tests FAILED"; tail -30 gpurun_out/ms_tests_$v.log; exit 1; }
  echo "MS=$v: $(tail -1 gpurun_out/ms_tests_$v.log)"
done
for r in 1 2; do for v in $1; do
  LBIC_DEC_MS=$v timeout -k 10 300 python3 bench.py --steps 16 --cpu-budget 0 --serial-steps 0 --substream-steps 0 \
      > gpurun_out/ms_$v.log 2>&1 || { tail -5 gpurun_out/ms_$v.log; exit 1; }
  echo "LBIC_DEC_MS=$v $(tail -1 gpurun_out/ms_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['quality']['enc_dec_bit_exact'], d['phases_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})")"
done; done
