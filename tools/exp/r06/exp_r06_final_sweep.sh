#!/bin/bash
# r06: at the final defaults (four batches per encoder pass): the encoder graph without its fork, and the first launch's
# footprint (12 / 14 workgroups per XCD slot instead of every CU)
set -eo pipefail
mkdir -p gpurun_out/r06
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
run() {   # tag, then extra args / env
  tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06/fs_${tag}.log 2>&1
  grep '^{' gpurun_out/r06/fs_${tag}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['kernels']['k_dec_team']['launch_windows_s'], d['kernels']['k_dec_team'].get('encoder_done_s'))"
}
for rep in 1 2; do
  run default_$rep $B
  run nofork_$rep LBIC_ENC_FORK=0 $B
  run fts12_$rep $B --first-team-size 12
  run fts14_$rep $B --first-team-size 14
done
