#!/bin/bash
# round 5, GPU call 26: the drain launch (16 teams, alone after the last encode) at two workgroups per CU -- teams of
# 32 workgroups, two teams' workgroups on every CU (latency of one team's operation hidden by the other's); team
# decode alone at WPC=2 and the bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for w in 2 1; do
  TEAMS=16 BATCH=32 WPC=$w SKIP_GRAPH=1 timeout -k 10 300 python3 -u tools/team_exp.py > $O/r05_c26_te_w$w.log 2>&1 || { echo "team_exp $w failed"; tail -5 $O/r05_c26_te_w$w.log; exit 5; }
  python3 -c "import json,sys; [print('team wpc', sys.argv[2], j['batches'], j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][0], j['op_us_mean']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r05_c26_te_w$w.log $w
done
for v in w2 w1 w2 w1; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --drain-wg-per-cu ${v#w} > $O/r05_c26_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c26_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c26_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], k['modes'])" $v
done
