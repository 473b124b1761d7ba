#!/bin/bash
# round 4, GPU call 12: no select between dependent MFMAs in the small-M chains (k_gemm_s, k_dec_team, k_dec_one: only the last
# fragment of a slice can be discarded), k_dec_one inputs-ready stamps: the whole GPU suite, single-image timing,
# team decode alone (8 batches), the driver's bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > $O/r04_c12_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r04_c12_tests.log; exit 3; }
tail -1 $O/r04_c12_tests.log
timeout -k 10 300 python3 -u tools/one_exp.py > $O/r04_c12_one.log 2>&1 || { echo "one_exp failed"; tail -10 $O/r04_c12_one.log; exit 4; }
grep '^{' $O/r04_c12_one.log
TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u tools/team_exp.py > $O/r04_c12_te.log 2>&1 || { echo "team_exp failed"; tail -5 $O/r04_c12_te.log; exit 5; }
python3 -c "import json,sys; [print('team', j['ms_per_batch'], j['bit_exact'], j['sampled_step_us'][:2], j['op_us_mean'], j['rans_done_us'][:4]) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r04_c12_te.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/r04_c12_bench.log 2>&1 || { echo "bench failed"; tail -20 $O/r04_c12_bench.log; exit 6; }
grep '^{' $O/r04_c12_bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['per_image']['dec_ms'], j['per_image']['enc_ms']); print(json.dumps(j['roofline']['per_kernel']))"
