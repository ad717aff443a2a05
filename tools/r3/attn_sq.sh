#!/bin/bash
# SQ counters (three separate --pmc passes, kernel-trace only) of the attention kernels at the decoder's
# T = 600 / D = 64 (tools/attn_one.py) and the encoder's T = 120 / D = 96 -> gpurun_out/$TAG/
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-attn_sq}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
P3="SQ_WAVES SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"
for shape in "600 64" "120 96"; do
  set -- $shape
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "attn_" --output-format csv -d $O/t$1_p$i -o run -- python3 $R/tools/attn_one.py $1 $2 5 > $O/t$1_p$i.log 2>&1; rc=$?
    echo "T=$1 pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/t$1_p$i.log; exit $rc; }
  done
done
timeout -k 10 120 python3 $R/tools/attn_one.py 600 64 20 > $O/time600.txt 2>&1 && cat $O/time600.txt
timeout -k 10 120 python3 $R/tools/attn_one.py 120 96 20 > $O/time120.txt 2>&1 && cat $O/time120.txt
