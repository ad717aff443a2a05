#!/bin/bash
# GEMM schedule replay of the bench step's launches (tools/r5/gemm_replay.py) -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5rp}; mkdir -p $O; cd $R
timeout -k 10 ${TO:-400} python -u tools/r5/gemm_replay.py ${LOG:-profiles/r05/gemm_log_parity.jsonl} ${ONLY:---only-bf16} --cfgs=${CFGS:--1,64,65,66,67,68,69} --out $O/replay.jsonl ${ARGS} > $O/replay.log 2>&1; rc=$?
tail -3 $O/replay.log; exit $rc
