#!/bin/bash
# round 5, GPU call 6 (HEAD after dropping k_gemm_t): the driver's bench command, the same command under rocprofv3
# --kernel-trace --stats (tools/gpu_round.sh: timed-region stats and wall occupancy per family), then the PMC traffic
# passes of both kernels at the headline's shapes (tools/pmc_round.sh -> pmc_traffic.json).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_round.sh r05c6 notests --steps 20 --warmup 5 || { echo "gpu_round failed"; tail -5 gpurun_out/bench_r05c6.log; exit 2; }
tail -1 gpurun_out/bench_r05c6.log | cut -c1-400
sed -n '/timed region/,$p' gpurun_out/kernel_stats_r05c6.txt
bash tools/pmc_round.sh || { echo "pmc failed"; exit 3; }
cat gpurun_out/pmc_headline.txt | head -60
