#!/bin/bash
# round 5, GPU call 25: the measurement set at the final HEAD (16 teams per launch, first launch on 12 of every XCD's
# CUs) -- PMC passes at the headline's shapes into profiles/pmc_traffic.json; the GPU suite, the driver's bench command
# and the same command under rocprofv3 --kernel-trace --stats (tools/gpu_round.sh); smoke(); configs 3-5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
bash tools/pmc_round.sh > $O/r05_c25_pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/r05_c25_pmc.log; exit 4; }
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json
grep -A3 '"k_dec_team"' $O/pmc_traffic.json | head -5; grep hbm_bytes_per_batch_step $O/pmc_traffic.json
bash tools/gpu_round.sh r05c25 tests --steps 20 --warmup 5 > $O/r05_c25_round.log 2>&1 || { echo "round failed"; tail -5 $O/r05_c25_round.log; tail -30 $O/gpu_tests_r05c25.log; exit 5; }
tail -1 $O/gpu_tests_r05c25.log
grep '^{' $O/bench_r05c25.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; r=j['roofline']; print('bench', j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], k['modes'], r['kernel'], r['bound'], r['frac'], r['traffic'], {a: (j.get(a) or {}).get('value') for a in ('eight_teams_per_launch','one_decode_in_flight','serial_schedule')})"
grep '^{' $O/bench_rocprof_r05c25.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench_rocprof', j['value'], j['roofline']['frac'], j['roofline']['avg_launch_us'])"
sed -n '/timed region only/,$p' $O/kernel_stats_r05c25.txt | head -8
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r05_c25_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/r05_c25_smoke.log; exit 6; }
tail -1 $O/r05_c25_smoke.log
bash tools/exp/r05/r05_cfg.sh r05c25 || exit 7
