#!/bin/bash
# (the k_gemm_c variants, LBIC_ENC_CFG 20-26, were removed after these measurements: DESIGN.md §4)
# round 3, GPU call 17: whole-K-per-wave encoder GEMM (k_gemm_c) configurations against the default k_gemm,
# encoder alone (tools/enc_exp.py: encode ms per 32-frame batch + digest of symbols / indexes / zhat)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for c in 0 20 21 22 23 24 25 26; do
  LBIC_ENC_CFG=$c timeout -k 10 120 python3 $R/tools/enc_exp.py > $O/r03_encc_cfg$c.log 2>&1 || { echo "cfg $c failed rc=$?"; tail -5 $O/r03_encc_cfg$c.log; exit 3; }
  tail -1 $O/r03_encc_cfg$c.log
done
