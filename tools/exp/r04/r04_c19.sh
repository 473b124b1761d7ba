#!/bin/bash
# round 4, GPU call 19: k_dec_one with the scale table in LDS, store stamps, rANS counters (main) vs the same with the
# first tile's weights read into registers before the waits (liblbic_wp.so), alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/r04_c19_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c19_tests.log; exit 3; }
tail -1 $O/r04_c19_tests.log
for v in main wp main wp; do
  unset LBIC_LIB_VARIANT
  if [ $v = wp ]; then export LBIC_LIB_VARIANT=wp; fi
  REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c19_one_$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c19_one_$v.log; exit 4; }
  echo "== $v"; grep '^{' $O/r04_c19_one_$v.log
done
