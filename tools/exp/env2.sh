set -eo pipefail
O=gpurun_out; mkdir -p $O
run() { local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 0 > $O/e2_$tag.log 2>&1
  grep '^{' $O/e2_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$tag', d['value'], d['ms_per_step'], d['phases_ms_per_step'], {n: (v['avg_span_us'], v['avg_launch_us']) for n, v in k.items()})"
}
run base X=1
run kgemm_dec LBIC_SMALL_MAX=0 LBIC_DEC_SMALL_MAX=0
run swz0 LBIC_ENC_SWZ=0
run cfg3_swz0 LBIC_ENC_CFG=3 LBIC_ENC_SWZ=0
run base2 X=1
run swz0b LBIC_ENC_SWZ=0
