#!/bin/bash
# same-box A/B of team-kernel variants: tools/exp/r06/exp_r06_ab.sh OUT REPS V1 V2 ... (cur = liblbic.so); team_exp at 16 teams
set -o pipefail
out=$1; reps=$2; shift 2
mkdir -p gpurun_out/r06
export SKIP_GRAPH=1 TEAMS=${TEAMS:-16}
for rep in $(seq $reps); do
  for v in "$@"; do
    if [ $v = cur ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
    echo "== $v rep $rep" >> $out
    timeout -k 10 200 python -u tools/team_exp.py 2>&1 | grep decoder >> $out || { echo "team $v failed"; exit 1; }
  done
done
echo done
