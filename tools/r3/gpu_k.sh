#!/bin/bash
# attention staging / max-fold: attention tests, timing at decoder + encoder shapes, SQ pass 2, glue tests, rows graph bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3k}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_step_glue_gpu.py -q --maxfail 6 --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error:|^E  " $O/tests.log | head -60; exit $rc; }
timeout -k 10 120 python3 tools/attn_one.py 600 64 20 > $O/time600.txt 2>&1 && cat $O/time600.txt
timeout -k 10 120 python3 tools/attn_one.py 120 96 20 > $O/time120.txt 2>&1 && cat $O/time120.txt
timeout -k 10 200 python -u tools/r3/rows_bench.py > $O/rows_bench.txt 2>&1; echo "rows rc=$?"; tail -9 $O/rows_bench.txt
cd /tmp && export TMPDIR=/tmp
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P2 --kernel-include-regex "attn_" --output-format csv -d $O/t600_p2 -o run -- python3 $R/tools/attn_one.py 600 64 5 > $O/t600_p2.log 2>&1; echo "pmc rc=$?"
