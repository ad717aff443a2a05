#!/bin/bash
# SQ / TCC counter passes over ONE replayed GEMM launch shape (tools/r5/gemm_replay.py --match), per schedule:
# MATCH="M,N,K,flags,act" CFGS="-1,96" -> gpurun_out/$TAG/pass*/ (each pass its own rocprofv3 run)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5pg}; mkdir -p $O; cd $R
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P5="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
have() { local out=""; for c in $1; do grep -qw "$c" $O/counters.txt && out="$out $c"; done; echo $out; }
i=0
for P0 in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i+1)); P=$(have "$P0"); echo "pass $i: $P"; [ -z "$P" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pass$i -o pmc --output-format csv -- python3 -u tools/r5/gemm_replay.py ${LOG:-profiles/r05/gemm_log_parity.jsonl} --match "$MATCH" --cfgs=${CFGS:--1,96} --plain ${REPS:-20} > $O/pass$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pass$i.log; exit 1; }
done
echo done
