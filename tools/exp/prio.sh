set -eo pipefail
O=gpurun_out; mkdir -p $O
python3 -c "import torch; print('priority range (least, greatest):', torch.cuda.Stream.priority_range())"
run() { local tag=$1; shift
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 "$@" > $O/prio_$tag.log 2>&1
  grep '^{' $O/prio_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'])"
}
run base
run dec_hi --dec-priority -1
run enc_lo --enc-priority 1
run dec_hi2 --dec-priority -2
run base2
