#!/bin/bash
# schedule sweep over the step's own GEMM calls (cfg x split-K)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3y}; mkdir -p $O; cd $R
timeout -k 10 900 python -u tools/r3/gemm_step_sweep.py > $O/sweep.jsonl 2> $O/sweep.err; rc=$?
tail -3 $O/sweep.err; wc -l $O/sweep.jsonl; exit $rc
