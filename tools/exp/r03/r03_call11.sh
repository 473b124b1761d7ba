#!/bin/bash
# round 3, GPU call 11: encoder tile configs not in the round-2 sweep (LBIC_ENC_CFG 2 = 16x32 / 8 waves / 2-k-block
# chunks), default twice for noise
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for c in 0 2 12 13 0; do
  LBIC_ENC_CFG=$c timeout -k 10 300 python -u tools/enc_exp.py > $O/r03_encexp2_cfg$c.log 2>&1 || exit 3
  echo "cfg $c $(grep encode_ms $O/r03_encexp2_cfg$c.log)"
done
