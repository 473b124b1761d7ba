#!/bin/bash
# round 5, GPU call 35: the final tree (workspace uploads on the caller's stream) -- GPU suite, smoke(), the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > $O/r05_c35_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05_c35_tests.log; exit 3; }
tail -1 $O/r05_c35_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r05_c35_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/r05_c35_smoke.log; exit 4; }
tail -1 $O/r05_c35_smoke.log
timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r05_c35_bench.log 2>&1 || { echo "bench failed"; tail -5 $O/r05_c35_bench.log; exit 5; }
grep '^{' $O/r05_c35_bench.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); k=j['kernels']['k_dec_team']; r=j['roofline']; print('bench', j['value'], j['ms_per_step'], k['launch_windows_s'], k['encoder_done_s'], k['modes'], r['kernel'], r['bound'], r['frac'], {a: (j.get(a) or {}).get('value') for a in ('eight_teams_per_launch','one_decode_in_flight','serial_schedule')}, j['config']['workload'][-160:])"
