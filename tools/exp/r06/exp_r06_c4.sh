#!/bin/bash
# r06 call 4: same-box A/B of team-kernel code variants (HEAD, option B, current) + encoder tile shapes (LBIC_ENC_CFG)
set -o pipefail
mkdir -p gpurun_out/r06
export SKIP_GRAPH=1 TEAMS=16
for rep in 1 2; do
  for v in abbase abB cur; do
    if [ $v = cur ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
    echo "== $v rep $rep" >> gpurun_out/r06/c4_ab.log
    timeout -k 10 200 python -u tools/team_exp.py 2>&1 | grep decoder >> gpurun_out/r06/c4_ab.log || { echo "team $v failed"; exit 1; }
  done
done
unset LBIC_LIB_VARIANT
for c in 0 1 2 3 4 5 6 7 0; do
  LBIC_ENC_CFG=$c timeout -k 10 120 python -u tools/enc_exp.py 2>&1 | grep encode_ms >> gpurun_out/r06/c4_enc.log || { echo "cfg $c failed: $?"; exit 1; }
done
echo done
