#!/bin/bash
# PMC passes at the headline's shapes, one counter group per rocprofv3 run (MI355X_MICROARCH.md): the encoder graph
# of one 32-frame 768x768 batch (tools/enc_exp.py) and a team decode launch of the headline's shape (tools/team_exp.py:
# 16 teams of 32 images, two per XCD); merged by
# tools/pmc_headline.py into gpurun_out/pmc_traffic.json (copy to profiles/ for bench.py).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/ef /tmp/ew /tmp/tf /tmp/tw /tmp/th
# the headline's encoder pass: --enc-pass 4 batches of 32 frames in one wavefront pass (ENC_BATCH)
export BATCH=${ENC_BATCH:-128} REPS=1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ef -o run -- python3 $R/tools/enc_exp.py > $O/pmc_enc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/ew -o run -- python3 $R/tools/enc_exp.py > $O/pmc_enc_write.log 2>&1
unset REPS
export TEAMS=16 BATCH=32 SKIP_GRAPH=1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/tf -o run -- python3 $R/tools/team_exp.py > $O/pmc_team_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/tw -o run -- python3 $R/tools/team_exp.py > $O/pmc_team_write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/th -o run -- python3 $R/tools/team_exp.py > $O/pmc_team_hit.log 2>&1
python3 $R/tools/pmc_summary.py $O/pmc_enc.json /tmp/ef /tmp/ew > $O/pmc_enc_summary.txt
python3 $R/tools/pmc_summary.py $O/pmc_team.json /tmp/tf /tmp/tw /tmp/th > $O/pmc_team_summary.txt
BATCH=${ENC_BATCH:-128} python3 $R/tools/pmc_headline.py $O/pmc_traffic.json $O/pmc_enc.json $O/pmc_team.json 16 96 96 32 > $O/pmc_headline.txt
echo pmc done
