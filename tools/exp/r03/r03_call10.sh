#!/bin/bash
# round 3, GPU call 10: team fast GEMM path extended to 1-3 k-blocks per K slice (B4 / KS3311 configs): team tests,
# configs 3-4, smoke
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "team" --timeout 300 --timeout-method thread > $O/r03_tests_v10.log 2>&1
rc=$?
tail -3 $O/r03_tests_v10.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; grep -E "FAILED|Error" $O/r03_tests_v10.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r03_smoke_v10.log 2>&1 || exit 2
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
timeout -k 10 300 $B --config B8_highrate --size 768 --height 512 --batch 3 --steps 12 --warmup 3 > $O/r03_cfg3_fast1.log 2>&1 || exit 3
timeout -k 10 400 $B --config B4_highrate --size 768 --batch 32 --steps 6 --warmup 3 > $O/r03_cfg4_fast1.log 2>&1 || exit 4
for f in $O/r03_cfg3_fast1.log $O/r03_cfg4_fast1.log; do
  grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels'].get('k_dec_team',{}); print('$(basename $f)', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['bpp'], d['quality']['enc_dec_bit_exact'], k.get('batch_decode_latency_ms'))"
done
cat $O/r03_smoke_v10.log | tail -2
