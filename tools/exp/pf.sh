#!/bin/bash
# Team decoder: weight tiles of the next GEMM requested at each team barrier (LBIC_TEAM_PF 0/1/2), decode alone
# (tools/team_exp.py, 8 batches in one launch) and the driver's bench command with encoder configs 6 / 7.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pf
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_team_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/team_tests.log 2>&1
LBIC_TEAM_PF=1 timeout -k 10 400 python -u -m pytest tests/test_team_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/team_tests_pf1.log 2>&1
for c in 7 12 13 14; do LBIC_ENC_CFG=$c timeout -k 10 120 python3 -u tools/enc_exp.py >> $O/enc.log 2>&1; done
for p in 0 1 2; do
  LBIC_TEAM_PF=$p TEAMS=8 timeout -k 10 200 python3 -u tools/team_exp.py > $O/team_$p.log 2>&1
  echo "pf $p $(grep ms_per_batch $O/team_$p.log | head -1 | cut -c1-200)" >> $O/summary.txt
done
for c in 7 12 13 14; do LBIC_ENC_CFG=$c timeout -k 10 120 python3 -u tools/enc_exp.py >> $O/enc.log 2>&1; done
for p in 0 1 2; do
  for c in 6 7; do
    LBIC_TEAM_PF=$p LBIC_ENC_CFG=$c timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 > $O/bench_${p}_$c.log 2>&1
    python3 - $O/bench_${p}_$c.log "pf $p cfg $c" >> $O/summary.txt <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{\"metric")][-1])
print(sys.argv[2], j["value"], j["ms_per_step"], j["phases_ms_per_step"])
PY
  done
done
cat $O/summary.txt
