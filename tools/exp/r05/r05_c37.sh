#!/bin/bash
# round 5, GPU call 37: where the 16-team decoder's wave time goes (SQ counters, one pass; team_exp: 16 teams of 32
# images alone) -- wave-parked / issue-stall / issuing quad-cycles and MFMA busy cycles per dispatch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/sq
TEAMS=16 BATCH=32 SKIP_GRAPH=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/sq -o run -- python3 $R/tools/team_exp.py > $O/r05_c37_sq.log 2>&1 || { echo "pmc failed"; tail -5 $O/r05_c37_sq.log; exit 3; }
python3 $R/tools/pmc_summary.py $O/r05_c37_sq.json /tmp/sq > $O/r05_c37_sq_summary.txt
python3 -c "
import json; d=json.load(open('$O/r05_c37_sq.json')); t=d.get('k_dec_team', {})
print({k: t[k] for k in sorted(t) if k.startswith('SQ') or k == 'dispatches'})
"
