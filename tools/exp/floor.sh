set -eo pipefail
O=gpurun_out; mkdir -p $O
for f in 0 41000 54000 82000 0; do
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 --enc-lds-floor $f > $O/floor_$f.log 2>&1
  grep '^{' $O/floor_$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('floor $f', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], d['kernels']['k_gemm']['avg_launch_us'])"
done
