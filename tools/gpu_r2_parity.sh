#!/bin/bash
# round 2: headline / long-form / synthesise / optimizer + accumulation parity tests (prints the measured errors)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r2_parity; mkdir -p $O
timeout -k 10 900 python -u -m pytest -s -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_encoder_ops_gpu.py::test_embedding_fwd_bitwise_bwd_deterministic tests/test_cfm_prep_gpu.py \
  tests/test_training_gpu.py tests/test_model_gpu.py tests/test_headline_gpu.py tests/test_longform_gpu.py \
  > $O/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|rel err|agreement|passed|failed" $O/tests.log | tail -60
exit $rc
