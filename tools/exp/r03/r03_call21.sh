#!/bin/bash
# round 3, GPU call 21: the team decoder's sparse rANS with its far-symbol table search in an LDS copy of the table
# image (LBIC_TEAM_SPARSE_LDS=1) against the global-memory search; per-rank rANS completion stamps of the sampled
# raster step (tools/team_exp.py rans_done_us); team GPU tests under the LDS variant; the driver's bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for v in 0 1; do
  LBIC_TEAM_SPARSE_LDS=$v TEAMS=8 SKIP_GRAPH=1 timeout -k 10 240 python3 -u $R/tools/team_exp.py > $O/r03_sparselds_$v.log 2>&1 || { echo "team_exp $v failed"; tail -5 $O/r03_sparselds_$v.log; exit 3; }
  python3 -c "import json,sys; [print(sys.argv[2], j['ms_per_batch'], j['bit_exact'], j['op_us_mean'], j['rans_done_us'], j['gemm_beside_rans_done_us']) for j in map(json.loads, [l for l in open(sys.argv[1]) if '\"decoder\": \"team\"' in l])]" $O/r03_sparselds_$v.log $v
done
LBIC_TEAM_SPARSE_LDS=1 timeout -k 10 300 python3 -u -m pytest tests/test_team_gpu.py tests/test_team_reference_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/r03_sparselds_tests.log 2>&1 || { echo "tests failed"; tail -20 $O/r03_sparselds_tests.log; exit 3; }
tail -2 $O/r03_sparselds_tests.log
for v in 0 1; do
  LBIC_TEAM_SPARSE_LDS=$v timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_benchsl_$v.txt 2> $O/r03_benchsl_$v.log || { echo "bench $v failed"; tail -5 $O/r03_benchsl_$v.log; exit 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_benchsl_$v.txt $v
done
# encoder tile shapes beside the team decoder (measured alone in rounds 2-3 only): 32x32 / 8 waves (cfg 13), 16x64 / 8 (cfg 12)
for c in 13 12; do
  LBIC_ENC_CFG=$c timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 5 --cpu-budget 0 --side-steps 0 --per-image 0 \
    > $O/r03_benchenc_$c.txt 2> $O/r03_benchenc_$c.log || { echo "bench enc $c failed"; tail -5 $O/r03_benchenc_$c.log; exit 3; }
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('enc_cfg', sys.argv[2], j['value'], j['ms_per_step'], j['phases_ms_per_step'], j['quality']['enc_dec_bit_exact'], j['kernels'].get('k_dec_team',{}).get('launch_ms_per_batch'))" $O/r03_benchenc_$c.txt $c
done
