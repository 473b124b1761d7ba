#!/bin/bash
# Sweep of the bench pipeline shape: "depth:gang[:steps[:enc_gang]]" (decoder handles in flight x batches per
# raster pass [x batches per encoder pass])
#   bash tools/ab_gang.sh "3:1 1:3 2:2 2:8:32:2"
set -o pipefail
mkdir -p gpurun_out
for spec in $1; do
  IFS=: read d g st eg <<< "$spec"
  st=${st:-12}; eg=${eg:-1}
  timeout -k 10 300 python3 bench.py --depth $d --gang $g --steps $st --enc-gang $eg --cpu-budget 0 --serial-steps 0 \
      --substream-steps 0 > gpurun_out/gang_${d}_${g}_${eg}.log 2>&1 || { tail -5 gpurun_out/gang_${d}_${g}_${eg}.log; exit 1; }
  echo "depth=$d gang=$g enc_gang=$eg $(tail -1 gpurun_out/gang_${d}_${g}_${eg}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['quality']['enc_dec_bit_exact'], d['phases_ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})")"
done
