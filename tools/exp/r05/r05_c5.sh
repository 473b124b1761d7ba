#!/bin/bash
# round 5, GPU call 5: the driver's bench with k_gemm_t v4 (default) and with k_gemm (LBIC_ENC_TILED=0) -- call 4's bench
# stopped at "corrupt bitstream" in the team decode; then SQ wave-state counters of the encoder alone, both kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/r05_c5_bench_t4.log 2>&1; echo "bench t4 rc=$?"
tail -1 $O/r05_c5_bench_t4.log | cut -c1-300
LBIC_ENC_TILED=0 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/r05_c5_bench_t0.log 2>&1; echo "bench t0 rc=$?"
tail -1 $O/r05_c5_bench_t0.log | cut -c1-300
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/ps*
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM"
P3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"
LBIC_ENC_TILED=4 timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d /tmp/ps1 -o run -- python3 $R/tools/enc_exp.py > $O/r05_c5_pmc1.log 2>&1 || exit 3
LBIC_ENC_TILED=0 timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d /tmp/ps2 -o run -- python3 $R/tools/enc_exp.py > $O/r05_c5_pmc2.log 2>&1 || exit 4
LBIC_ENC_TILED=4 timeout -s KILL 150 rocprofv3 --pmc $P3 --output-format csv -d /tmp/ps3 -o run -- python3 $R/tools/enc_exp.py > $O/r05_c5_pmc3.log 2>&1 || exit 5
python3 $R/tools/pmc_summary.py $O/r05_c5_pmc_t4.json /tmp/ps1 /tmp/ps3 > /dev/null
python3 $R/tools/pmc_summary.py $O/r05_c5_pmc_t0.json /tmp/ps2 > /dev/null
python3 - $O/r05_c5_pmc_t4.json $O/r05_c5_pmc_t0.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    for k in ("k_gemm_t", "k_gemm", "k_gemm_s"):
        if k in d:
            print(f.split('/')[-1], k, {c: round(v, 1) for c, v in d[k].items()})
PY
