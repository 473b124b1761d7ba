set -eo pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 --depth 2 --gang 2 > $O/g2d2.log 2>&1
grep '^{' $O/g2d2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('d2', d['value'], d['ms_per_step']); g=d['gang_schedule']; print('gang2 x depth2', g['value'], g['ms_per_step'], g['phases_ms_per_step'])"
timeout -k 10 400 python3 -u bench.py --cpu-budget 0 --side-steps 0 --depth 4 --gang 2 > $O/g2d4.log 2>&1
grep '^{' $O/g2d4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('d4', d['value'], d['ms_per_step']); g=d['gang_schedule']; print('gang2 x depth2 (second run)', g['value'], g['ms_per_step'], g['phases_ms_per_step'])"
