#!/bin/bash
# round 3, GPU call 13: narrowed code transport with the copy stream on its own hardware queue (only the streams the
# team schedule uses are created), A/B x2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for nc in 0 1 0 1; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --narrow-codes $nc > $O/r03_bench13_nc${nc}_$RANDOM.log 2>&1 || exit 2
done
for f in $O/r03_bench13_nc*.log; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$(basename $f)', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['enc_dec_bit_exact'])
"; done
exit 0
