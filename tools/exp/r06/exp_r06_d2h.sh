#!/bin/bash
# r06: the driver's bench command with the encoder's D2H copies on a copy stream (default) vs on the encoder stream
set -eo pipefail
mkdir -p gpurun_out/r06
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
for rep in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 $B --d2h-stream $v > gpurun_out/r06/d2h_${v}_rep$rep.log 2>&1
    grep '^{' gpurun_out/r06/d2h_${v}_rep$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('d2h=$v rep $rep', d['value'], d['ms_per_step'], d['kernels']['k_dec_team']['launch_windows_s'], d['kernels']['k_dec_team'].get('encoder_done_s'))"
  done
done
