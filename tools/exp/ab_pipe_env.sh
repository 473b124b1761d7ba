#!/bin/bash
# A/B of a liblbic environment toggle on the default pipelined bench (gang 16, enc-gang 4), two rounds each:
#   bash tools/ab_pipe_env.sh VAR "v1 v2"
set -o pipefail
VAR=$1; VALS=$2
mkdir -p gpurun_out
for r in 1 2; do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python3 bench.py --cpu-budget 0 --serial-steps 0 --substream-steps 0 \
      > gpurun_out/pab_${VAR}_${v}.log 2>&1 || { tail -5 gpurun_out/pab_${VAR}_${v}.log; exit 1; }
  echo "$VAR=$v $(tail -1 gpurun_out/pab_${VAR}_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['quality']['enc_dec_bit_exact'], d['phases_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})")"
done; done
