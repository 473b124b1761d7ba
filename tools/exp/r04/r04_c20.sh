#!/bin/bash
# round 4, GPU call 20: k_dec_one pacing (LBIC_ONE_PACE, an A/B switch) against none, then the round's final
# tools/gpu_round.sh: the whole GPU suite, the driver's bench and its rocprofv3 kernel-trace stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in 0 250 0 300; do
  LBIC_ONE_PACE=$v REPS=5 timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c20_one_p$v.log 2>&1 || { echo "one_exp $v failed"; tail -10 $O/r04_c20_one_p$v.log; exit 4; }
  echo "== pace $v"; grep '"decoder": "one"' $O/r04_c20_one_p$v.log
done
bash tools/gpu_round.sh r04c20 tests --steps 20 --warmup 5 || { echo "gpu_round failed"; tail -30 $O/gpu_tests_r04c20.log; tail -20 $O/bench_r04c20.log; exit 5; }
tail -1 $O/gpu_tests_r04c20.log
grep '^{' $O/bench_r04c20.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['per_image']['dec_ms'], j['per_image']['dec_team_ms'], j['per_image']['enc_ms']); print(json.dumps(j['roofline']['per_kernel'])); print(json.dumps(j['cpu_baseline']))"
head -30 $O/kernel_stats_r04c20.txt
