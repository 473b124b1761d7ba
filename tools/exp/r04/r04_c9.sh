#!/bin/bash
# round 4, GPU call 9: k_dec_one with sentinel polling (one lane per workgroup polls the op's latest input until it
# shows up) and predicated granule loads: GPU tests, then single-image timing + stamps with the sentinel on and off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -s -m gpu --timeout 180 --timeout-method thread > $O/r04_c9_one.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c9_one.log; exit 3; }
tail -1 $O/r04_c9_one.log
for S in 1 0; do
  LBIC_ONE_SENT=$S timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c9_exp_s$S.log 2>&1 || { echo "one_exp failed"; tail -10 $O/r04_c9_exp_s$S.log; exit 4; }
  echo "sentinel $S"; grep '^{' $O/r04_c9_exp_s$S.log
done
