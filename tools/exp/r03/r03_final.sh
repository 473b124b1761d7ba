#!/bin/bash
# round 3 final measurement: the GPU suite, the driver's bench command, the same command under rocprofv3
# --kernel-trace --stats (tools/gpu_round.sh), then the team decoder's PMC traffic passes (tools/team_pmc.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_round.sh ${1:-r03v1} tests --steps 20 --warmup 5 || exit 1
bash tools/team_pmc.sh || exit 2
python3 tools/pmc_merge.py profiles/pmc_traffic.json gpurun_out/team_pmc.json gpurun_out/pmc_traffic_r03.json > /dev/null
tail -3 gpurun_out/gpu_tests_${1:-r03v1}.log
grep '^{' gpurun_out/bench_${1:-r03v1}.log | cut -c1-400
cat gpurun_out/kernel_stats_${1:-r03v1}.txt | head -20
