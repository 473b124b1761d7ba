#!/bin/bash
# round 4, GPU call 26: the committed final tree -- smoke() and the whole GPU suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_c26_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/r04_c26_smoke.log; exit 2; }
tail -2 $O/r04_c26_smoke.log
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/r04_c26_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c26_tests.log; exit 3; }
tail -1 $O/r04_c26_tests.log
REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c26_one.log 2>&1 || { echo "one_exp failed"; exit 4; }
grep '"decoder"' $O/r04_c26_one.log
