set -eo pipefail
O=gpurun_out; mkdir -p $O
for v in new prev new prev; do
  if [ $v = prev ]; then B=_bench_prev.py; else B=bench.py; fi
  timeout -k 10 300 python3 -u $B --cpu-budget 0 --side-steps 0 > $O/ovl_$v.log 2>&1
  grep '^{' $O/ovl_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['quality']['enc_dec_bit_exact'])"
done
