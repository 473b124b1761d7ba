#!/bin/bash
# Encoder graph fork (LBIC_ENC_FORK=1: context net || transform branches, join at the quantising GEMM) vs one chain:
# encoder alone (tools/enc_exp.py digests must agree), the GPU parity tests with the fork, and the driver's bench.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/fork
mkdir -p $O
cd $R
for f in 0 1; do LBIC_ENC_FORK=$f timeout -k 10 120 python3 -u tools/enc_exp.py >> $O/enc.log 2>&1; done
LBIC_ENC_FORK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests_fork.log 2>&1
for f in 0 1 0 1; do
  LBIC_ENC_FORK=$f timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 > $O/bench_$f.log 2>&1
  python3 - $O/bench_$f.log "fork $f" >> $O/summary.txt <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{\"metric")][-1])
print(sys.argv[2], j["value"], j["ms_per_step"], j["phases_ms_per_step"])
PY
done
grep -v amdgpu.ids $O/enc.log; tail -1 $O/tests_fork.log; cat $O/summary.txt
