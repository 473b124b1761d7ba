#!/bin/bash
# round 4, GPU call 15: k_dec_one with the scale indexes from ctx3's epilogue and barrier-free stamps (main library) vs
# the same with row-0-only A-fragment loads (liblbic_ra.so) and with the far-waiter gate (LBIC_ONE_GATE=3), alternated; single-image tests on the main library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/r04_c15_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c15_tests.log; exit 3; }
tail -1 $O/r04_c15_tests.log
for v in main ra gate main ra gate; do
  unset LBIC_LIB_VARIANT LBIC_ONE_GATE
  if [ $v = ra ]; then export LBIC_LIB_VARIANT=ra; fi
  if [ $v = gate ]; then export LBIC_ONE_GATE=3; fi
  REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c15_one_$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c15_one_$v.log; exit 4; }
  echo "== $v"; grep '^{' $O/r04_c15_one_$v.log
done
