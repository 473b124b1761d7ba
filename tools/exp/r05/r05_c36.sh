#!/bin/bash
# round 5, GPU call 36: config 3's shard with the sub-stream leg (concurrent first decodes that capture row graphs) at
# the final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0 --config B8_highrate --size 768 --height 512 --batch 3 --steps 16 --warmup 4 --substream-steps 16 > $O/r05_c36_cfg3_$i.log 2>&1 || { echo "cfg3 failed"; tail -5 $O/r05_c36_cfg3_$i.log; exit 3; }
grep '^{' $O/r05_c36_cfg3_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('substream_format') or {}; print('cfg3', d['value'], d['quality']['enc_dec_bit_exact'], s.get('value'), s.get('enc_dec_bit_exact'))"
done
