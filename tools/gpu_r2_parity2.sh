#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r2_parity2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -s -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_training_gpu.py tests/test_model_gpu.py::test_synthesise_vs_reference tests/test_headline_gpu.py \
  > $O/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|rel err|agreement|largest|passed|failed|^E  .*Error" $O/tests.log | cut -c1-400 | tail -60
exit $rc
