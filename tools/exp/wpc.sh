#!/bin/bash
# Team decode launches with two workgroups per CU (LBC_OPT_TEAM_WG_PER_CU=2, teams of 64) vs one: team tests, decode
# alone (tools/team_exp.py, 8 batches per launch), the driver's bench with the drain launch at 1 / 2 per CU; then the
# XCD-aware encoder tile order (LBIC_ENC_SWZ) A/B.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wpc
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_team_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/team_tests.log 2>&1
for w in 1 2; do
  WPC=$w TEAMS=8 SKIP_GRAPH=1 timeout -k 10 200 python3 -u tools/team_exp.py > $O/team_$w.log 2>&1
  echo "wpc $w $(grep ms_per_batch $O/team_$w.log | head -1 | cut -c1-200)" >> $O/summary.txt
done
bench() {
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 "$@" > $O/b.log 2>&1
  python3 - $O/b.log "$*" >> $O/summary.txt <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{\"metric")][-1])
print(sys.argv[2], j["value"], j["ms_per_step"], j["phases_ms_per_step"], j["roofline"]["kernel"], j["roofline"]["avg_launch_us"])
PY
}
bench --drain-wg-per-cu 1
bench --drain-wg-per-cu 2
bench --drain-wg-per-cu 1
bench --drain-wg-per-cu 2
for f in 0 1; do LBIC_ENC_SWZ=$f timeout -k 10 120 python3 -u tools/enc_exp.py >> $O/enc_swz.log 2>&1; done
LBIC_ENC_SWZ=1 bench
LBIC_ENC_SWZ=1 bench
grep -v amdgpu.ids $O/enc_swz.log; tail -1 $O/team_tests.log; cat $O/summary.txt
