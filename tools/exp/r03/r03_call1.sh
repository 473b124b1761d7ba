#!/bin/bash
# round 3, GPU call 1: the GPU suite (new: team vs the reference's decompress(), column-split teams, timeout fallback,
# config 1 through main.py, the N-rank bench path), then decode-only and headline A/B of the team geometry.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/r03_tests_v1.log 2>&1
rc=$?
tail -30 $O/r03_tests_v1.log
[ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
SKIP_GRAPH=1 TEAMS=8 LBIC_TEAM_XS=0 timeout -k 10 300 python -u tools/team_exp.py > $O/r03_teamexp_xs0.log 2>&1 &&
SKIP_GRAPH=1 TEAMS=8 LBIC_TEAM_XS=1 timeout -k 10 300 python -u tools/team_exp.py > $O/r03_teamexp_xs1.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --team-xs 0 --cpu-budget 0 --side-steps 0 > $O/r03_bench_xs0.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --team-xs 1 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r03_bench_xs1.log 2>&1
rc2=$?
grep -h '"decoder"' $O/r03_teamexp_xs*.log | cut -c1-300
echo "rc=$rc rc2=$rc2"
exit $rc2
