#!/bin/bash
# HBM traffic of the conv/linear GEMM launches (register-staged, LDS-DMA and split-K combine kernels) per launch, as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes:
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (they do not fit one TCC pass), FETCH_SIZE doubled
# on gfx950, per dispatch, kernels restricted to conv_gemm_kernel.  Output: gpurun_out/$1/
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-pmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "conv_gemm_kernel|conv_gemm_glds_kernel|splitk_epilogue_kernel" --output-format csv -d $O/fetch -o run -- python3 $R/tools/pmc_traffic.py $O/algo.json > $O/fetch.log 2>&1; rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/fetch.log; exit $rc; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "conv_gemm_kernel|conv_gemm_glds_kernel|splitk_epilogue_kernel" --output-format csv -d $O/write -o run -- python3 $R/tools/pmc_traffic.py $O/algo2.json > $O/write.log 2>&1; rc=$?; echo "write rc=$rc"; exit $rc
