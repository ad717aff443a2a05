#!/bin/bash
# per-shape GEMM and wgrad tables of the step (eager, HIP events), for planning
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3n}; mkdir -p $O; cd $R
timeout -k 10 200 python -u tools/step_gemms.py > $O/gemms.txt 2>&1; echo "gemms rc=$?"; head -40 $O/gemms.txt
timeout -k 10 200 python -u tools/step_wgrads.py > $O/wgrads.txt 2>&1; echo "wgrads rc=$?"; head -40 $O/wgrads.txt
