#!/bin/bash
# round 4, GPU call 24: k_dec_one polls that read the clock (s_memrealtime) only every 16th round, like the failure
# word (liblbic_tm.so), against main, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
LBIC_LIB_VARIANT=tm timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/r04_c24_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c24_tests.log; exit 3; }
tail -1 $O/r04_c24_tests.log
for v in main tm main tm; do
  unset LBIC_LIB_VARIANT
  if [ $v = tm ]; then export LBIC_LIB_VARIANT=tm; fi
  REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c24_one_$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c24_one_$v.log; exit 4; }
  echo "== $v"; grep '^{' $O/r04_c24_one_$v.log
done
