set -eo pipefail
O=gpurun_out; mkdir -p $O
LBIC_ENC_CFG=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/kw_tests.log 2>&1
tail -1 $O/kw_tests.log
run() { local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --cpu-budget 0 --side-steps 2 > $O/kw_$tag.log 2>&1
  grep '^{' $O/kw_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$tag', d['value'], d['ms_per_step'], d['phases_ms_per_step'], 'serial', d['serial_schedule']['phases_ms_per_step'], {n: (v['avg_span_us'], v['avg_launch_us']) for n, v in k.items()})"
}
run cfg0 LBIC_ENC_CFG=0
run cfg4 LBIC_ENC_CFG=4
run cfg5 LBIC_ENC_CFG=5
run cfg6 LBIC_ENC_CFG=6
run cfg7 LBIC_ENC_CFG=7
run cfg8 LBIC_ENC_CFG=8
