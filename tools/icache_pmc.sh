#!/bin/bash
# Instruction-cache counters of a 16-team k_dec_team launch (tools/team_exp.py) and of the encoder graph
# (tools/enc_exp.py): one rocprofv3 --pmc pass each (MI355X_MICROARCH.md), summaries under gpurun_out/.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${PMC_TAG:-r06}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/pmc_avail.txt 2>&1 || true
rm -rf /tmp/ic /tmp/iw /tmp/ie
export TEAMS=16 BATCH=32 SKIP_GRAPH=1
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d /tmp/ic -o run -- python3 $R/tools/team_exp.py > $O/pmc_icache_team.log 2>&1 || echo "team pass failed: $?"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH --output-format csv -d /tmp/iw -o run -- python3 $R/tools/team_exp.py > $O/pmc_ifetch_team.log 2>&1 || echo "team ifetch pass failed: $?"
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d /tmp/ie -o run -- python3 $R/tools/enc_exp.py > $O/pmc_icache_enc.log 2>&1 || echo "enc pass failed: $?"
python3 $R/tools/pmc_summary.py $O/pmc_icache.json /tmp/ic /tmp/iw /tmp/ie > $O/pmc_icache_summary.txt
echo pmc done
