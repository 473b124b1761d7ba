set -eo pipefail
O=gpurun_out; mkdir -p $O
run() { local tag=$1; shift
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 "$@" > $O/wk_$tag.log 2>&1
  grep '^{' $O/wk_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], d['quality']['enc_dec_bit_exact'])"
}
run w4 --workers 4
run w4_f41 --workers 4 --enc-lds-floor 41000
run d3_f41 --enc-lds-floor 41000
run d3_f36 --enc-lds-floor 36000
run d3_f46 --enc-lds-floor 46000
run w3 --workers 3
run w4_s40 --workers 4 --steps 40
run d3 
