#!/bin/bash
# r06: the first decode launch's footprint at the driver's 32 batches (16 teams, two per XCD slot): --first-team-size
set -eo pipefail
mkdir -p gpurun_out/r06
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
for rep in 1 2; do
  for v in 8 10 12 14 16; do
    timeout -k 10 300 $B --first-team-size $v > gpurun_out/r06/fts_${v}_rep$rep.log 2>&1
    grep '^{' gpurun_out/r06/fts_${v}_rep$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fts=$v rep $rep', d['value'], d['ms_per_step'], d['kernels']['k_dec_team']['launch_windows_s'], d['kernels']['k_dec_team'].get('encoder_done_s'))"
  done
done
