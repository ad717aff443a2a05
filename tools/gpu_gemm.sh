#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 200 python tools/gemm_bench.py bf16 > $O/gemm_bf16.log 2>&1; rc=$?; cat $O/gemm_bf16.log | grep shape; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $O/pmc_gemm -o p1 -- python3 $R/tools/gemm_bench.py bf16 > $O/pmc1.log 2>&1; echo pmc1 rc=$?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_gemm -o p2 -- python3 $R/tools/gemm_bench.py bf16 > $O/pmc2.log 2>&1; echo pmc2 rc=$?
ls $O/pmc_gemm
