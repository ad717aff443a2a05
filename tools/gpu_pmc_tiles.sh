#!/bin/bash
# SQ counters for conv_gemm_glds at two schedules (64x64 vs 160x128) on the 19200 x 256 x 768 conv, bf16 A
R=${GRAFT_REPO_ROOT:-$(pwd)}
for c in 44 48; do
  bash $R/tools/pmc_sq.sh conv_gemm_glds tools/gemm_one.py conv3_full_256 $c 5 bf16 || exit 1
  python3 $R/tools/pmc_sq_summary.py $R/gpurun_out/pmc_sq > $R/gpurun_out/pmc_tiles_$c.txt
  grep -h "^ok" $R/gpurun_out/pmc_sq/p1.log >> $R/gpurun_out/pmc_tiles_$c.txt
  rm -rf $R/gpurun_out/pmc_sq
done
