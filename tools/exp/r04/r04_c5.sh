#!/bin/bash
# round 4, GPU call 5: the tree with the ring opt-in (default off), the encoder's k_gemm launch duration from in-kernel
# stamps (earliest start -> latest end over the XCDs) in the bench line, team spread 1/2/4/8: the whole GPU suite; batch-1
# team decode at each spread beside the graph decoder; the driver's bench command and the same command under rocprofv3
# (k_gemm per-launch duration, line vs trace); configs 3-5 (config 3 in both formats).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/r04_c5_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/r04_c5_tests.log; exit 3; }
tail -1 $O/r04_c5_tests.log
for P in 1 2 4 8; do
  LBIC_TEAM_SPREAD=$P BATCH=1 TEAMS=1 timeout -k 10 200 python3 -u tools/team_exp.py > $O/r04_c5_b1_s$P.log 2>&1 || { echo "b1 spread $P failed"; tail -5 $O/r04_c5_b1_s$P.log; exit 4; }
  python3 -c "import json,sys; [print('spread $P', j.get('decoder'), j.get('ms_per_batch'), j.get('bit_exact'), j.get('sampled_step_us', [None])[:2]) for j in map(json.loads, [l for l in open(sys.argv[1]) if l.startswith('{') and 'decoder' in l])]" $O/r04_c5_b1_s$P.log
done
bash tools/gpu_round.sh r04c5 notests --steps 20 --warmup 5 || { echo "gpu_round failed"; exit 5; }
grep '^{' $O/bench_r04c5.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['per_image']); print(json.dumps(j['roofline']['per_kernel'])); print(json.dumps(j['kernels']['k_gemm']))"
cat $O/kernel_stats_r04c5.txt
bash tools/exp/r04/r04_cfg.sh c5
