#!/bin/bash
# round 4, GPU call 23: the round's final state -- single-image timing and stamps, then tools/gpu_round.sh: the whole
# GPU suite, the driver's bench and its rocprofv3 kernel-trace stats (same command).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c23_one.log 2>&1 || { echo "one_exp failed"; tail -10 $O/r04_c23_one.log; exit 4; }
grep '"decoder"' $O/r04_c23_one.log
bash tools/gpu_round.sh r04c23 tests --steps 20 --warmup 5 || { echo "gpu_round failed"; tail -30 $O/gpu_tests_r04c23.log; tail -20 $O/bench_r04c23.log; exit 5; }
tail -1 $O/gpu_tests_r04c23.log
grep '^{' $O/bench_r04c23.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['per_image']['dec_ms'], j['per_image']['dec_team_ms'], j['per_image']['enc_ms']); print(json.dumps(j['roofline'])); print(json.dumps(j['cpu_baseline']))"
head -12 $O/kernel_stats_r04c23.txt
grep -A8 "timed region" $O/kernel_stats_r04c23.txt
