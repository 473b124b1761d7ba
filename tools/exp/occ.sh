#!/bin/bash
# Encoder GEMM residency beside the team decoder: LBIC_ENC_CFG 0 (88 VGPRs), 4 (CH=1, <=64), 5 (CH=2, <=80),
# 6 (CH=1, 70): encoder alone (tools/enc_exp.py) and the driver's bench command (--steps 20 --warmup 5).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/occ
mkdir -p $O
cd $R
[ -n "$TESTS" ] && timeout -k 10 400 python -u -m pytest tests/test_team_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/team_tests.log 2>&1
for c in ${CFGS:-0 4 5 6}; do
  LBIC_ENC_CFG=$c timeout -k 10 120 python3 -u tools/enc_exp.py >> $O/enc.log 2>&1
done
for c in ${CFGS:-0 4 5 6}; do
  LBIC_ENC_CFG=$c timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 > $O/bench_$c.log 2>&1
  python3 - $O/bench_$c.log $c >> $O/summary.txt <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{\"metric")][-1])
print(sys.argv[2], j["value"], j["ms_per_step"], j["phases_ms_per_step"], j["roofline"]["avg_launch_us"], j["roofline"]["frac"])
PY
done
cat $O/enc.log $O/summary.txt
