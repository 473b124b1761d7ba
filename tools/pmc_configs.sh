#!/bin/bash
# PMC traffic at the launch shapes of BASELINE configs 3-5 (bench.py --config ..., tools/config_lines.sh): one
# FETCH_SIZE and one WRITE_SIZE rocprofv3 pass (MI355X_MICROARCH.md) over a team decode launch of the config's shape
# (tools/team_exp.py, ONE=1) and over the config's encoder graph (tools/enc_exp.py); merged by tools/pmc_configs.py
# into gpurun_out/pmc_configs.json (copy its entries into profiles/pmc_traffic.json "configs" for bench.py).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_cfg
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() {   # tag, frames per encoder pass, then env assignments for the config
  tag=$1; ENCB=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf /tmp/pc_${tag}_team_$c /tmp/pc_${tag}_enc_$c
    env "$@" ONE=1 SKIP_GRAPH=1 timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d /tmp/pc_${tag}_team_$c -o run -- python3 $R/tools/team_exp.py > $O/${tag}_team_$c.log 2>&1
    # the encoder at the bench's pass shape: --enc-pass 4 batches in one wavefront pass (ENCB frames)
    env "$@" REPS=1 BATCH=$ENCB timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d /tmp/pc_${tag}_enc_$c -o run -- python3 $R/tools/enc_exp.py > $O/${tag}_enc_$c.log 2>&1
  done
  python3 $R/tools/pmc_summary.py $O/${tag}_team.json /tmp/pc_${tag}_team_FETCH_SIZE /tmp/pc_${tag}_team_WRITE_SIZE > $O/${tag}_team_summary.txt
  python3 $R/tools/pmc_summary.py $O/${tag}_enc.json /tmp/pc_${tag}_enc_FETCH_SIZE /tmp/pc_${tag}_enc_WRITE_SIZE > $O/${tag}_enc_summary.txt
  echo "$tag done"
}
# config 3 shard: 3 frames of 768x512 per batch, two batches per team, 16 batches (8 teams) per launch
run B8_highrate 12 CONFIG=B8_highrate SIZE=768 HEIGHT=512 BATCH=3 TB=2 TEAMS=8
# config 4: 32 frames of 768x768 per batch, one per team, 16 teams per launch
run B4_highrate 128 CONFIG=B4_highrate SIZE=768 BATCH=32 TB=1 TEAMS=16
# config 5: 8 frames of 2048x2048 per batch, two batches per team, 16 batches (8 teams) per launch
run B16_lowrate 32 CONFIG=B16_lowrate SIZE=2048 BATCH=8 TB=2 TEAMS=8
python3 $R/tools/pmc_configs.py $R/gpurun_out/pmc_configs.json $O > $O/merge.txt
echo pmc configs done
