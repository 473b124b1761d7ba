#!/bin/bash
# PMC passes over the team decoder (tools/team_exp.py, 8 batches of 32 B8_lowrate 768x768 frames in one k_dec_team
# launch, run twice): fabric-side read / write bytes and L2 hit rate per launch.  Outputs under gpurun_out/.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/tf /tmp/tw /tmp/th
export TEAMS=8 SKIP_GRAPH=1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/tf -o run -- python3 $R/tools/team_exp.py > $O/team_pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/tw -o run -- python3 $R/tools/team_exp.py > $O/team_pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/th -o run -- python3 $R/tools/team_exp.py > $O/team_pmc_hit.log 2>&1
python3 $R/tools/pmc_summary.py $O/team_pmc.json /tmp/tf /tmp/tw /tmp/th > $O/team_pmc_summary.txt
grep -A12 k_dec_team $O/team_pmc.json | head -30
