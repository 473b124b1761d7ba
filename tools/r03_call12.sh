#!/bin/bash
# round 3, GPU call 12: narrowed code transport (int16 / uint8 on a copy stream) A/B at the driver's command; the
# N-rank bench test; config 5 with the round-3 team decoder
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "bench_two_ranks" --timeout 300 --timeout-method thread > $O/r03_tests_v12.log 2>&1 || { tail -30 $O/r03_tests_v12.log; exit 1; }
tail -2 $O/r03_tests_v12.log
for nc in 1 0; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --narrow-codes $nc > $O/r03_bench_nc${nc}_$RANDOM.log 2>&1 || exit 2
done

for f in $O/r03_bench_nc*.log $O/r03_cfg5_v12.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$(basename $f)', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['enc_dec_bit_exact'])
"; done
