set -eo pipefail
O=gpurun_out; mkdir -p $O
run() { local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 --workers 4 > $O/ec_$tag.log 2>&1
  grep '^{' $O/ec_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['phases_ms_per_step'], d['roofline']['avg_launch_us'], d['kernels']['k_gemm']['avg_launch_us'])"
}
run cfg0 LBIC_ENC_CFG=0
run cfg1 LBIC_ENC_CFG=1
run cfg2 LBIC_ENC_CFG=2
run cfg3 LBIC_ENC_CFG=3
run swz0 LBIC_ENC_SWZ=0
run cfg0b LBIC_ENC_CFG=0
