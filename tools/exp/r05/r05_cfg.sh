#!/bin/bash
# round 5: BASELINE configs 3-5 at HEAD (call 8: one batch per team; call 18: two) (config 5 at its recalibrated 0.12 bpp point), with config 3 in BOTH bitstream formats (VERDICT r3 item 3 -> r4 item 6): the 3-frame
# 768x512 shard of one GPU (of 8) and all 24 frames on one GPU, each with the reference-format headline schedule and an
# opt-in sub-stream leg (--substream-steps: per-block-row streams, wavefront decode).  usage: r04_cfg.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-x}
mkdir -p $O
cd $R
B="python3 -u bench.py --cpu-budget 0 --side-steps 0 --per-image 0"
run() {  # name, timeout, args...
  local f=$1 t=$2; shift 2
  timeout -k 10 $t $B "$@" > $O/${f}_$TAG.log 2>&1 || { echo "$f failed"; tail -5 $O/${f}_$TAG.log; return 3; }
  grep '^{' $O/${f}_$TAG.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('substream_format') or {}
print('$f', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['bpp'], d['quality']['enc_dec_bit_exact'],
      '| rows:', s.get('value'), s.get('ms_per_step'), s.get('bpp'), s.get('enc_dec_bit_exact'), s.get('phases_ms_per_step'))"
}
run cfg3_shard 300 --config B8_highrate --size 768 --height 512 --batch 3 --steps 16 --warmup 4 --substream-steps 16 && \
run cfg3_all24 400 --config B8_highrate --size 768 --height 512 --batch 24 --steps 8 --warmup 3 --substream-steps 8 --team-batches 1 && \
run cfg4 400 --config B4_highrate --size 768 --batch 32 --steps 6 --warmup 3 --team-batches 1 && \
run cfg5 400 --config B16_lowrate --size 2048 --batch 8 --steps 6 --warmup 3
