#!/bin/bash
# XCD-aware encoder tile order (LBIC_ENC_SWZ=1: XCD bid%8 gets a contiguous run of row-major tiles) vs plain order,
# encoder alone (digests must agree), parity tests with it, and the driver's bench.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/swz
mkdir -p $O
cd $R
for f in 0 1; do LBIC_ENC_SWZ=$f timeout -k 10 120 python3 -u tools/enc_exp.py >> $O/enc.log 2>&1; done
LBIC_ENC_SWZ=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_fork.log 2>&1
for f in 0 1 0 1; do
  LBIC_ENC_SWZ=$f timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 > $O/bench_$f.log 2>&1
  python3 - $O/bench_$f.log "swz $f" >> $O/summary.txt <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{\"metric")][-1])
print(sys.argv[2], j["value"], j["ms_per_step"], j["phases_ms_per_step"])
PY
done
grep -v amdgpu.ids $O/enc.log; tail -1 $O/tests_fork.log; cat $O/summary.txt
