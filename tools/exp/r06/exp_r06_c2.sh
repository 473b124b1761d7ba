#!/bin/bash
# r06 call 2: instruction-cache counters and team-decoder timing, HEAD vs the smaller-code variant (liblbic_icb.so)
set -eo pipefail
mkdir -p gpurun_out/r06
export SKIP_GRAPH=1
TEAMS=16 timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c2_te16_base.log 2>&1
LBIC_LIB_VARIANT=icb TEAMS=16 timeout -k 10 200 python -u tools/team_exp.py > gpurun_out/r06/c2_te16_icb.log 2>&1
LBIC_LIB_VARIANT=icb timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_team_gpu.py tests/test_team_reference_gpu.py > gpurun_out/r06/c2_tests_icb.log 2>&1
PMC_TAG=r06/c2_base bash tools/icache_pmc.sh
LBIC_LIB_VARIANT=icb PMC_TAG=r06/c2_icb bash tools/icache_pmc.sh
echo done
