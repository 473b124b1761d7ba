#!/bin/bash
# r06 call 12: per-wave A-issue / A-arrival stamps (diag), then the encoder launch accounting
set -eo pipefail
mkdir -p gpurun_out/r06
SKIP_GRAPH=1 TEAMS=16 LBIC_LIB_VARIANT=tdiag timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c12_te16_diag.log 2>&1
bash tools/exp/r06/exp_r06_enc.sh
echo done
