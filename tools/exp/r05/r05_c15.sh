#!/bin/bash
# round 5, GPU call 15: the measurement set at the two-batch-team HEAD -- PMC passes at the headline's shapes (encoder
# graph; 8 teams of 64 images) into profiles/pmc_traffic.json, then the GPU suite, the driver's bench command and the
# same command under rocprofv3 --kernel-trace --stats (tools/gpu_round.sh), then smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
bash tools/pmc_round.sh > $O/r05_c15_pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/r05_c15_pmc.log; exit 4; }
cp $O/pmc_traffic.json $R/profiles/pmc_traffic.json
cat $O/pmc_headline.txt | head -40
bash tools/gpu_round.sh r05c15 tests --steps 20 --warmup 5 > $O/r05_c15_round.log 2>&1 || { echo "round failed"; tail -5 $O/r05_c15_round.log; tail -30 $O/gpu_tests_r05c15.log; exit 5; }
tail -3 $O/gpu_tests_r05c15.log
grep '^{' $O/bench_r05c15.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench', j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['kernels']['k_dec_team']['launch_windows_s'], j['kernels']['k_dec_team']['encoder_done_s'], j['roofline']['kernel'], j['roofline']['bound'], j['roofline']['frac'], j['roofline']['traffic'])"
grep '^{' $O/bench_rocprof_r05c15.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('bench_rocprof', j['value'], j['roofline']['frac'], j['roofline']['avg_launch_us'])"
head -30 $O/kernel_stats_r05c15.txt
cd $R && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r05_c15_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/r05_c15_smoke.log; exit 6; }
tail -1 $O/r05_c15_smoke.log
