#!/bin/bash
# same-box A/B of single-image decode (tools/one_exp.py) between library variants: OUT REPS CONFIG V1 V2 ...
set -o pipefail
out=$1; reps=$2; cfg=$3; shift 3
mkdir -p gpurun_out/r06
for rep in $(seq $reps); do
  for v in "$@"; do
    if [ $v = cur ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
    echo "== $v rep $rep" >> $out
    CONFIG=$cfg REPS=3 timeout -k 10 200 python -u tools/one_exp.py 2>&1 | grep '"decoder": "one"' >> $out || { echo "one $v failed"; exit 1; }
  done
done
echo done
