#!/bin/bash
# round 3, GPU call 16: what bounds k_gemm (encoder alone) and k_dec_team (8 batches alone): SQ wave states, MFMA busy,
# TA busy / stalls, L1->L2 read latency (separate --pmc passes, each within the per-block slot limits)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/ps*
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM"
P2="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TA_TCP_STATE_READ_sum GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d /tmp/ps1 -o run -- python3 $R/tools/enc_exp.py > $O/r03_pmc_enc1.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d /tmp/ps2 -o run -- python3 $R/tools/enc_exp.py > $O/r03_pmc_enc2.log 2>&1 || exit 4
export TEAMS=8 SKIP_GRAPH=1
timeout -s KILL 200 rocprofv3 --pmc $P1 --output-format csv -d /tmp/ps3 -o run -- python3 $R/tools/team_exp.py > $O/r03_pmc_team1.log 2>&1 || exit 5
timeout -s KILL 200 rocprofv3 --pmc $P2 --output-format csv -d /tmp/ps4 -o run -- python3 $R/tools/team_exp.py > $O/r03_pmc_team2.log 2>&1 || exit 6
python3 $R/tools/pmc_summary.py $O/r03_pmc_bound_enc.json /tmp/ps1 /tmp/ps2 > /dev/null
python3 $R/tools/pmc_summary.py $O/r03_pmc_bound_team.json /tmp/ps3 /tmp/ps4 > /dev/null
python3 - $O/r03_pmc_bound_enc.json $O/r03_pmc_bound_team.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    for k in ("k_gemm<16,32,8,1,1>", "k_dec_team<false>"):
        if k in d:
            print(f.split('/')[-1], k, {c: round(v, 1) for c, v in d[k].items()})
PY
