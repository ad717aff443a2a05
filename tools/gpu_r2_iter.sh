#!/bin/bash
# One iteration: the whole GPU suite, then an interleaved step A/B over env settings (tools/gpu_ab3.sh).
# Usage: gpu_r2_iter.sh TAG SETTING... (each setting = comma-separated env assignments, DUMMY=0 = defaults)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; shift; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|^FAILED|Error" $O/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab3.sh "$@"
