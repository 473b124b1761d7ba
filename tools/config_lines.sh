#!/bin/bash
# Bench lines for BASELINE.json configs 3-5 at their frame sizes, one GPU's shard each (outputs under gpurun_out/);
# 16 batches each, so every decode launch has >= 8 teams (every XCD decodes):
#   3  B8_highrate N1152M128, Kodak-24 sharded over 8 GPUs: 3 frames of 768x512 per GPU (and the whole 24 on one)
#   4  B4_highrate N512M96 on one GPU: batches of 32 synthetic 768x768 frames
#   5  B16_lowrate N1280M192, 2048x2048 frames over 8 GPUs: batches of 8 frames per GPU
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-x}
mkdir -p $O
cd $R
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
timeout -k 10 300 $B --config B8_highrate --size 768 --height 512 --batch 3 --steps 16 --warmup 3 > $O/cfg3_shard_$TAG.log 2>&1
timeout -k 10 300 $B --config B8_highrate --size 768 --height 512 --batch 24 --steps 8 --warmup 3 > $O/cfg3_all24_$TAG.log 2>&1
timeout -k 10 500 $B --config B4_highrate --size 768 --batch 32 --steps 16 --warmup 3 > $O/cfg4_$TAG.log 2>&1
timeout -k 10 500 $B --config B16_lowrate --size 2048 --batch 8 --steps 16 --warmup 3 > $O/cfg5_$TAG.log 2>&1
for f in cfg3_shard cfg3_all24 cfg4 cfg5; do
  grep '^{' $O/${f}_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels'].get('k_dec_team', {}); print('$f', d['value'], d['unit'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['bpp'], d['quality']['enc_dec_bit_exact'], k.get('launch_windows_s'), k.get('modes'), d['roofline']['frac'], d['roofline']['traffic_source'])"
done
