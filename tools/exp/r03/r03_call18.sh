#!/bin/bash
# (the k_gemm_c variants, LBIC_ENC_CFG 20-26, were removed after these measurements: DESIGN.md §4)
# round 3, GPU call 18: encoder launch times by GEMM shape for k_gemm (cfg 0) and k_gemm_c (cfg 20, 22); then the
# encoder alone at capped residency (LDS floor: 3 / 2 workgroups of 8 waves per CU = 6 / 4 waves per SIMD)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in 0 20 22; do
  rm -rf /tmp/et$c
  LBIC_ENC_CFG=$c timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/et$c -o run -- python3 $R/tools/enc_exp.py > $O/r03_encc_trace$c.log 2>&1 || exit 3
  python3 $R/tools/enc_shapes.py $(find /tmp/et$c -name "*kernel_trace.csv" | head -1) > $O/r03_encc_shapes$c.txt || exit 4
  head -12 $O/r03_encc_shapes$c.txt
done
for f in 53000 80000; do
  LDS_FLOOR=$f timeout -k 10 120 python3 $R/tools/enc_exp.py > $O/r03_enc_floor$f.log 2>&1 || exit 5
  tail -1 $O/r03_enc_floor$f.log
done
