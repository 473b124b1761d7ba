#!/bin/bash
# round 4, GPU call 10: k_dec_one with exact K slices for K = 768 / 1152, the rANS table image in the stream
# workgroup's LDS, rANS sub-stamps; the sentinel removed.  GPU tests, single-image timing + stamps, and the experiment
# build with the first tile's weights prefetched into registers (liblbic_wpre.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_one_gpu.py -x -v -s -m gpu --timeout 180 --timeout-method thread > $O/r04_c10_one.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c10_one.log; exit 3; }
tail -1 $O/r04_c10_one.log
for V in base wpre; do
  if [ $V = base ]; then E=""; else E="LBIC_LIB_VARIANT=$V"; fi
  env $E timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c10_exp_$V.log 2>&1 || { echo "one_exp $V failed"; tail -10 $O/r04_c10_exp_$V.log; exit 4; }
  echo "$V"; grep '^{' $O/r04_c10_exp_$V.log
done
