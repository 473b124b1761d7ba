#!/bin/bash
# round 3, GPU call 4: team GEMM load order (A first, (A, W) interleaved) vs the round-2 order (liblbic_wfirst.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "team" --timeout 300 --timeout-method thread > $O/r03_tests_v4.log 2>&1
rc=$?
tail -3 $O/r03_tests_v4.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
for v in new wfirst; do
  if [ $v = new ]; then unset LBIC_LIB_VARIANT; else export LBIC_LIB_VARIANT=$v; fi
  SKIP_GRAPH=1 TEAMS=8 timeout -k 10 300 python -u tools/team_exp.py > $O/r03_teamexp_$v.log 2>&1 || exit 3
done
unset LBIC_LIB_VARIANT
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r03_bench_new.log 2>&1 &&
LBIC_LIB_VARIANT=wfirst timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r03_bench_wfirst.log 2>&1
rc2=$?
for v in new wfirst; do grep -h '"decoder"' $O/r03_teamexp_$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', d['ms_per_batch'], d['sampled_step_us'][:3], d['op_us_team0'])"; done
for f in $O/r03_bench_new.log $O/r03_bench_wfirst.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d['phases_ms_per_step'])
"; done
exit $rc2
