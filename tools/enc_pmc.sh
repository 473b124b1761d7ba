#!/bin/bash
# PMC passes over the encoder alone (tools/enc_exp.py: one 32-frame B8_lowrate 768x768 batch, 4 compressions), for
# the GEMM variant LBIC_ENC_TILED selects: MFMA busy, LDS bank conflicts, wave cycles.  Outputs under gpurun_out/.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
V=${1:-3}
mkdir -p $O
export TMPDIR=/tmp LBIC_ENC_TILED=$V
cd /tmp
rm -rf /tmp/ep1_$V /tmp/ep2_$V
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --output-format csv -d /tmp/ep1_$V -o run -- python3 $R/tools/enc_exp.py > $O/enc_pmc1_$V.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VALU --output-format csv -d /tmp/ep2_$V -o run -- python3 $R/tools/enc_exp.py > $O/enc_pmc2_$V.log 2>&1
python3 $R/tools/pmc_summary.py $O/enc_pmc_$V.json /tmp/ep1_$V /tmp/ep2_$V > /dev/null
python3 - $O/enc_pmc_$V.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("k_gemm", "k_gemm_t", "k_gemm_s"):
    if k in d:
        print(k, {c: round(v, 1) for c, v in d[k].items() if c != "dispatches"}, "dispatches", d[k]["dispatches"])
PY
