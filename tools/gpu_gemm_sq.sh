#!/bin/bash
# SQ counter passes for conv_gemm tile configs on one shape: bash tools/gpu_gemm_sq.sh SHAPE CFG...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/gemm_sq; mkdir -p $O; cd $R
SHAPE=${1:-conv3_full_256}; shift
for c in "$@"; do
  bash tools/pmc_sq.sh conv_gemm tools/gemm_one.py $SHAPE $c 3 || exit 1
  python tools/pmc_sq_summary.py $R/gpurun_out/pmc_sq > $O/sq_${SHAPE}_cfg$c.txt; rm -rf $R/gpurun_out/pmc_sq
done
cat $O/sq_${SHAPE}_cfg*.txt
