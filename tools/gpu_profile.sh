#!/bin/bash
# PMC passes for roofline.traffic (FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs: MI355X_MICROARCH.md
# "rocprofv3 PMC slots"): the headline's launch shapes (32-row decoder raster steps, the encoder's wavefront
# steps over one 32-frame batch) on 64x64 frames -- a raster step has 32 rows whatever the frame size, so the
# per-launch shapes equal the 768x768 run's -- merged by tools/pmc_summary.py into profiles/pmc_traffic.json,
# which bench.py reads.  Outputs under gpurun_out/.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/pf /tmp/pw
ARGS="--size 64 --steps 2 --warmup 1 --cpu-budget 0 --side-steps 0"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- \
    python3 $R/bench.py $ARGS > $O/prof_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- \
    python3 $R/bench.py $ARGS > $O/prof_write.log 2>&1
python3 $R/tools/pmc_summary.py $O/pmc_traffic.json /tmp/pf /tmp/pw > $O/pmc_summary.txt
echo done
