#!/bin/bash
# Round 4: the bf16x3 / parity-policy tests and the default bench line (parity headline) -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4prec}; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_weight_split_gpu.py tests/test_headline_gpu.py tests/test_longform_gpu.py::test_train_forward_512x4096_bucketed tests/test_model_gpu.py::test_decoder_more_than_eight_resnets_vs_oracle tests/test_dp_gpu.py tests/test_dp_multirank_gpu.py tests/test_training_gpu.py -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|rel err|agreement" $O/tests.log | tail -60
[ $rc -ne 0 ] && { grep -E "^E  " $O/tests.log | head -30; }
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err; rc2=$?
echo "bench rc=$rc2"; [ $rc2 -ne 0 ] && { tail -20 $O/bench.err; exit $rc2; }
python tools/r4/bench_summary.py $O/bench.json
exit $rc
