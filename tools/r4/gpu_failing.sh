#!/bin/bash
# round 4: the graph-mode failures of r4s1 with the in-kernel split sums on and off (MTTS_WGRAD_FUSED_SUM)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4fail}; mkdir -p $O; cd $R
T="tests/test_training_gpu.py::test_graph_gradients_equal_eager_over_replays tests/test_training_gpu.py::test_decoder_prefetch_matches_inline tests/test_training_gpu.py::test_accumulate_grad_batches_2_vs_torch tests/test_dp_gpu.py tests/test_headline_gpu.py::test_headline_b4_vs_reference"
for F in 1 0; do
  MTTS_WGRAD_FUSED_SUM=$F timeout -k 10 400 python -u -m pytest $T -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/fused$F.log 2>&1; rc=$?
  echo "fused=$F rc=$rc"; tail -3 $O/fused$F.log; grep -E "^FAILED|^E  .{0,160}" $O/fused$F.log | head -8
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
done
exit 0
