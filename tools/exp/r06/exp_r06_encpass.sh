#!/bin/bash
# r06: two 32-frame batches per encoder wavefront pass (--enc-pass 2) vs one, the driver's command otherwise
set -eo pipefail
mkdir -p gpurun_out/r06
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
for rep in 1 2; do
  for v in 2 4 1; do
    timeout -k 10 300 $B --enc-pass $v > gpurun_out/r06/encpass_${v}_rep$rep.log 2>&1
    grep '^{' gpurun_out/r06/encpass_${v}_rep$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('enc_pass=$v rep $rep', d['value'], d['ms_per_step'], d['kernels']['k_dec_team']['launch_windows_s'], d['kernels']['k_dec_team'].get('encoder_done_s'))"
  done
done
