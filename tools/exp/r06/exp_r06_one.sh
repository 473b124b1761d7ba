#!/bin/bash
# r06: k_dec_one with the layer-0 cache (KS3311) -- the single-image tests, then per-image decode of one 768x768 frame
# for B4_highrate and B8_lowrate (k_dec_one vs the row graphs, stamps of the middle step)
set -eo pipefail
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_one_gpu.py > gpurun_out/r06/one_tests.log 2>&1
CONFIG=B4_highrate REPS=2 timeout -k 10 200 python -u tools/one_exp.py > gpurun_out/r06/one_b4.log 2>&1
CONFIG=B8_lowrate REPS=2 timeout -k 10 100 python -u tools/one_exp.py > gpurun_out/r06/one_b8.log 2>&1
echo done
