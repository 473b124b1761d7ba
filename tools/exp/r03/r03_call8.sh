#!/bin/bash
# round 3, GPU call 8: encoder k-loop pipeline depth (LBIC_ENC_CFG 16-19: 2-3 k-blocks in flight per wave) vs default
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for c in 0 16 17 18 19 0; do
  LBIC_ENC_CFG=$c timeout -k 10 300 python -u tools/enc_exp.py > $O/r03_encexp_cfg$c.log 2>&1 || exit 3
  echo "cfg $c $(grep encode_ms $O/r03_encexp_cfg$c.log)"
done
