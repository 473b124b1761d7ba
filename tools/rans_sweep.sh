#!/bin/bash
# k_rans_decode (LDS table image) vs k_rans_decode_sparse (centre-interval fast path) on synthetic streams of
# 32 images x 96 symbols per step, over the symbol spread (value ~ N(0, spread x table scale)): the crossover
# sets LBIC_RANS_SPARSE_BPS.  Output: gpurun_out/rans_sweep.log
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
B=$R/learned-block-based-image-compression_amd/csrc/build/rans_bench
mkdir -p $R/gpurun_out
for sp in 0.05 0.2 0.4 0.8 1.2 3.0; do
  for v in 0 1; do
    timeout -k 5 60 $B 32 96 0 63 $v $sp
  done
done > $R/gpurun_out/rans_sweep.log 2>&1
for v in 0 1; do timeout -k 5 60 $B 32 96 0 20 $v 0.3; done >> $R/gpurun_out/rans_sweep.log 2>&1
cat $R/gpurun_out/rans_sweep.log
