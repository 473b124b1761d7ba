#!/bin/bash
# r06: decode launch groups at the driver's 32 batches with the first launch on every CU (--first-team-size 16)
set -eo pipefail
mkdir -p gpurun_out/r06
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0 --first-team-size 16"
for rep in 1 2; do
  for v in 16,16 16,8,8 8,8,16 12,12,8 8,16,8; do
    timeout -k 10 300 $B --team-sizes $v > gpurun_out/r06/grp_${v}_rep$rep.log 2>&1
    grep '^{' gpurun_out/r06/grp_${v}_rep$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('groups=$v rep $rep', d['value'], d['ms_per_step'], d['kernels']['k_dec_team']['launch_windows_s'], d['kernels']['k_dec_team'].get('encoder_done_s'))"
  done
done
