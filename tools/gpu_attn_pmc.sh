#!/bin/bash
# attention kernels alone: timing + kernel trace + PMC passes -> gpurun_out/$1/
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-apmc}; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/attn_one.py 600 64 20 > $O/one.txt 2>&1 || exit 1
timeout -k 10 120 python3 $R/tools/attn_one.py 300 64 20 >> $O/one.txt 2>&1 || exit 1
cat $O/one.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/attn_one.py 600 64 5 > /dev/null 2>$O/kt.err || exit 1
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $O/pmc$i -o run -- python3 $R/tools/attn_one.py 600 64 2 > /dev/null 2>$O/pmc$i.err || { echo "pmc$i failed"; tail -3 $O/pmc$i.err; exit 1; }
done
echo done
