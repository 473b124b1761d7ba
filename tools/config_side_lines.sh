#!/bin/bash
# BASELINE configs 3-5, the legs config_lines.sh skips: the opt-in sub-stream format for config 3 (3-frame shard and
# all 24 on one GPU) and eval_model's per-image path (batch 1: compress() then decompress() of ONE frame) of configs
# 3, 4 and 5 -- short runs (2 batches of the main schedule).  Outputs under gpurun_out/.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-x}
mkdir -p $O
cd $R
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --warmup 2 --steps 2"
timeout -k 10 300 $B --config B8_highrate --size 768 --height 512 --batch 3 --substream-steps 16 --per-image 1 > $O/cfg3_side_$TAG.log 2>&1
timeout -k 10 300 $B --config B8_highrate --size 768 --height 512 --batch 24 --substream-steps 8 --per-image 0 > $O/cfg3_all24_side_$TAG.log 2>&1
timeout -k 10 300 $B --config B4_highrate --size 768 --batch 32 --per-image 1 > $O/cfg4_side_$TAG.log 2>&1
timeout -k 10 300 $B --config B16_lowrate --size 2048 --batch 8 --per-image 1 > $O/cfg5_side_$TAG.log 2>&1
for f in cfg3_side cfg3_all24_side cfg4_side cfg5_side; do
  grep '^{' $O/${f}_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('substream_format') or {}; p=d.get('per_image') or {}; print('$f', 'substream', s.get('value'), s.get('ms_per_step'), 'per_image', p.get('enc_ms'), p.get('dec_ms'), p.get('dec_path'), p.get('enc_dec_bit_exact'))"
done
