#!/bin/bash
# round 5, GPU call 17: the driver's bench command (default side legs, now with one_batch_per_team) and the drain
# launch at two workgroups per CU (--drain-wg-per-cu 2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 > $O/r05_c17_bench_def.log 2>&1 || { echo "bench def failed"; tail -5 $O/r05_c17_bench_def.log; exit 6; }
grep '^{' $O/r05_c17_bench_def.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench def', j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], {a: j[a]['value'] if j.get(a) else None for a in ('one_batch_per_team','one_decode_in_flight','serial_schedule')}, j['per_image'])"
for v in w2 w1 w2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 --drain-wg-per-cu ${v#w} > $O/r05_c17_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 $O/r05_c17_bench_$v.log; exit 6; }
  grep '^{' $O/r05_c17_bench_$v.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; print('bench', sys.argv[1], j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'])" $v
done
