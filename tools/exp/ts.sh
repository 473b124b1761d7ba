#!/bin/bash
# Team size beside the encoder: LBIC_TEAM_S caps the workgroups per team (32 = one per CU of an XCD); smaller teams
# leave whole CUs to the encoder.  Driver's bench command, two runs each.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ts
mkdir -p $O
cd $R
bench() {
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 > $O/b.log 2>&1
  python3 - $O/b.log "S=$LBIC_TEAM_S" >> $O/summary.txt <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{\"metric")][-1])
print(sys.argv[2], j["value"], j["ms_per_step"], j["phases_ms_per_step"], j["roofline"]["kernel"], j["roofline"]["avg_launch_us"])
PY
}
for s in 32 28 24 20 32 28 24 20; do LBIC_TEAM_S=$s bench; done
cat $O/summary.txt
