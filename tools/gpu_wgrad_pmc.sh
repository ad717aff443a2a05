#!/bin/bash
# wgrad operand-storage A/B: graph timings, then SQ counters per instantiation
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/wgpmc; mkdir -p $O
timeout -k 10 120 python3 $R/tools/wgrad_store_ab.py conv3 > $O/times.txt 2>&1 || { tail $O/times.txt; exit 1; }
timeout -k 10 120 python3 $R/tools/wgrad_store_ab.py lin_256_1024 >> $O/times.txt 2>&1 || exit 1
cat $O/times.txt | grep ok
bash $R/tools/pmc_sq.sh conv_wgrad_kernel tools/wgrad_store_ab.py conv3 || exit 1
python3 $R/tools/pmc_sq_summary.py $R/gpurun_out/pmc_sq > $O/sq.txt
rm -rf $R/gpurun_out/pmc_sq
