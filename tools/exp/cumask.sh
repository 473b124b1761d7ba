set -eo pipefail
O=gpurun_out; mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 "$@" > $O/cm_$tag.log 2>&1
  grep '^{' $O/cm_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'])"
}
run d3 --depth 3
run d3_e50 --depth 3 --enc-cu-frac 0.5
run d3_e25 --depth 3 --enc-cu-frac 0.25
run d3_e75 --depth 3 --enc-cu-frac 0.75
run d4_e50 --depth 4 --enc-cu-frac 0.5
run d4_e50_d50 --depth 4 --enc-cu-frac 0.5 --dec-cu-frac 0.5
run d3_e50_d75 --depth 3 --enc-cu-frac 0.5 --dec-cu-frac 0.75
