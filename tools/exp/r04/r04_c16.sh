#!/bin/bash
# round 4, GPU call 16: k_dec_one stamps kept in registers until after each publish (no stamp traffic in the waits);
# the far-waiter gate (LBIC_ONE_GATE=3) against none, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/r04_c16_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c16_tests.log; exit 3; }
tail -1 $O/r04_c16_tests.log
for v in main gate3 main gate3 gate2; do
  unset LBIC_ONE_GATE
  if [ $v = gate3 ]; then export LBIC_ONE_GATE=3; fi
  if [ $v = gate2 ]; then export LBIC_ONE_GATE=2; fi
  REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c16_one_$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c16_one_$v.log; exit 4; }
  echo "== $v"; grep '^{' $O/r04_c16_one_$v.log
done
