#!/bin/bash
# round 3, GPU call 6: configs 3-4 (weight-stream-bound raster steps: the KS3311 context layer 1 is a 5-tap GEMM of
# K = 5 C1) with column-split teams and cross-team step alignment
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "team" --timeout 300 --timeout-method thread > $O/r03_tests_v6.log 2>&1
rc=$?
tail -3 $O/r03_tests_v6.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; grep -E "FAILED|Error" $O/r03_tests_v6.log | head; exit $rc; }
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
for cfg in "0 0" "1 0" "1 2"; do
  set -- $cfg
  LBIC_TEAM_ALIGN=$2 timeout -k 10 300 $B --team-xs $1 --config B8_highrate --size 768 --height 512 --batch 3 --steps 12 --warmup 3 > $O/r03_cfg3_xs$1_al$2.log 2>&1 || exit 3
  LBIC_TEAM_ALIGN=$2 timeout -k 10 400 $B --team-xs $1 --config B4_highrate --size 768 --batch 32 --steps 6 --warmup 3 > $O/r03_cfg4_xs$1_al$2.log 2>&1 || exit 4
done
for f in $O/r03_cfg3_xs*.log $O/r03_cfg4_xs*.log; do
  grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels'].get('k_dec_team',{}); print('$(basename $f)', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['bpp'], d['quality']['enc_dec_bit_exact'], k.get('batch_decode_latency_ms'), k.get('column_split'))"
done
