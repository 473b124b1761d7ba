#!/bin/bash
# r06: encoder tile shapes at the headline's 128-frame passes (LBIC_ENC_TILE 0: 16x32, 1: 32x32, 2: 16x64), encoder
# alone (tools/enc_exp.py), then the driver's bench command with the best two
set -eo pipefail
mkdir -p gpurun_out/r06
for rep in 1 2; do
  for t in 0 1 2; do
    echo "== tile $t rep $rep" >> gpurun_out/r06/tile_enc.log
    LBIC_ENC_TILE=$t BATCH=128 REPS=3 timeout -k 10 200 python -u tools/enc_exp.py 2>&1 | grep encode_ms >> gpurun_out/r06/tile_enc.log
  done
done
cat gpurun_out/r06/tile_enc.log
