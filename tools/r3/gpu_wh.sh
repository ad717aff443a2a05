#!/bin/bash
# 96-row LDS-DMA tiles: sweep the step's decoder-size GEMM calls over the LDS-DMA configs (no split)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wh}; mkdir -p $O; cd $R
SWEEP_GLDS=32-51 SWEEP_SPLITS=1 SWEEP_REG=1 SWEEP_MIN_ROWS=9600 timeout -k 10 900 python -u tools/r3/gemm_step_sweep.py > $O/sweep.jsonl 2> $O/sweep.err; rc=$?
tail -3 $O/sweep.err; wc -l $O/sweep.jsonl; exit $rc
