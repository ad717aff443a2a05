#!/bin/bash
# rows GEMM (time MLP): kernel trace of the graph-replayed fwd+bwd, SQ counters
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3o}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/r3/rows_bench.py > $O/trace.log 2>&1; echo "trace rc=$?"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_WAVES SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "rows_gemm" --output-format csv -d $O/p$i -o run -- python3 $R/tools/r3/rows_bench.py > $O/p$i.log 2>&1; echo "pass $i rc=$?"
done
