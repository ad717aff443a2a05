#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r2_parity3; mkdir -p $O
timeout -k 10 600 python -u -m pytest -s -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_training_gpu.py::test_clip_adamw_matches_torch \
  > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|rel err|agreement|largest|passed|failed|^E  .*Error" $O/tests.log | cut -c1-400 | tail -40
rc1=$rc
timeout -k 10 300 python -u tools/adamw_debug.py > $O/adamw.log 2>&1; grep -E " p:" $O/adamw.log | cut -c1-200
exit $rc1
