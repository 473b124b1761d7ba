#!/bin/bash
# round 4, GPU call 21: k_dec_one with the rANS centre-symbol runs on the vector ALU (state in a VGPR, intervals as
# broadcast LDS reads) -- main -- against the scalar runs (liblbic_prev.so), alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/r04_c21_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c21_tests.log; exit 3; }
tail -1 $O/r04_c21_tests.log
for v in main prev main prev; do
  unset LBIC_LIB_VARIANT
  if [ $v = prev ]; then export LBIC_LIB_VARIANT=prev; fi
  REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c21_one_$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c21_one_$v.log; exit 4; }
  echo "== $v"; grep '^{' $O/r04_c21_one_$v.log
done
