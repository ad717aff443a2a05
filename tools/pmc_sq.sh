#!/bin/bash
# SQ counter passes (separate --pmc runs, kernel-trace only) for the kernels matching $1, over the
# command given after it (python script + args): gpurun_out/pmc_sq/<pass>/...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmc_sq; mkdir -p $O
RE=$1; shift
SCRIPT=$1; shift
case "$SCRIPT" in /*) ;; *) SCRIPT=$R/$SCRIPT ;; esac
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS"
P3="SQ_WAVES SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$RE" --output-format csv -d $O/p$i -o run -- python3 "$SCRIPT" "$@" > $O/p$i.log 2>&1 && grep -q "^ok" $O/p$i.log || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
