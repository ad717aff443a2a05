#!/bin/bash
# round 5: MAS / split-K (bf16x6) / DP tests after the ADVICE fixes, MAS PMC traffic, forced-DP step profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5c3}; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests/test_mas_gpu.py tests/test_weight_split_gpu.py tests/test_dp_gpu.py tests/test_dp_multirank_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-r5c3}/pmcmas bash tools/r5/pmc_mas.sh || exit 1
MTTS_FORCE_DP=1 TAG=${TAG:-r5c3}/dpprof bash tools/r5/gpu_prof.sh || exit 1
TAG=${TAG:-r5c3}/prof bash tools/r5/gpu_prof.sh || exit 1
