#!/bin/bash
# round 3, GPU call 3: encoder pass size (frames per wavefront pass) alone, and the headline with one- and two-batch
# encoder passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "dense_two or step_alignment" --timeout 300 --timeout-method thread > $O/r03_tests_v3.log 2>&1
rc=$?
tail -3 $O/r03_tests_v3.log
[ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
for b in 32 64 128; do
  BATCH=$b timeout -k 10 300 python -u tools/enc_exp.py > $O/r03_encexp_b$b.log 2>&1 || exit 4
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r03_bench_ep1.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --enc-pass 2 > $O/r03_bench_ep2.log 2>&1
rc2=$?
cat $O/r03_encexp_b*.log | grep encode
for f in $O/r03_bench_ep1.log $O/r03_bench_ep2.log; do python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['ms_per_step'], d['phases_ms_per_step'])
"; done
exit $rc2
