#!/bin/bash
# round 3, GPU call 5: cross-operation register prefetch (LBIC_TEAM_XPF) correctness and A/B; configs 3-5 at their
# operating points
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "team" --timeout 300 --timeout-method thread > $O/r03_tests_v5.log 2>&1
rc=$?
tail -3 $O/r03_tests_v5.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; grep -E "FAILED|Error" $O/r03_tests_v5.log | head; exit $rc; }
for x in 0 1; do
  SKIP_GRAPH=1 TEAMS=8 LBIC_TEAM_XPF=$x timeout -k 10 300 python -u tools/team_exp.py > $O/r03_teamexp_xpf$x.log 2>&1 || exit 3
done
for x in 0 1; do
  LBIC_TEAM_XPF=$x timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 > $O/r03_bench_xpf$x.log 2>&1 || exit 4
done
for x in 0 1; do grep -h '"decoder"' $O/r03_teamexp_xpf$x.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('xpf$x', d['ms_per_batch'], d['sampled_step_us'][:3], d['op_us_team0'])"; done
for x in 0 1; do python3 -c "
import json
for l in open('$O/r03_bench_xpf$x.log'):
    if l.startswith('{'):
        d=json.loads(l); print('bench xpf$x', d['value'], d['ms_per_step'], d['phases_ms_per_step'])
"; done
bash tools/config_lines.sh r03v1
