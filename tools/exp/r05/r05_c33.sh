#!/bin/bash
# round 5, GPU call 33: the headline's 16-batch launch in the full-size tests (decode == encode at 16 x 32 x 768^2; the
# reference's full-frame fixture inside a 16-team launch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest "tests/test_fullsize_gpu.py::test_team_full_size_roundtrip" tests/test_team_reference_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -s > $O/r05_c33_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c33_tests.log; exit 3; }
grep -E "PASSED|FAILED|passed|failed|bits per symbol" $O/r05_c33_tests.log | tail -20
