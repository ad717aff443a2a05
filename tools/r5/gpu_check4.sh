#!/bin/bash
# round 5: weight-stationary GEMM + 16-byte epilogue: GEMM / decoder-op / weight-split / headline tests, then the
# bench line (TESTS= overrides the test list)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5c4}; mkdir -p $O; cd $R
T=${TESTS:-tests/test_gemm_wreg_gpu.py tests/test_decoder_ops_gpu.py tests/test_weight_split_gpu.py tests/test_headline_gpu.py}
timeout -k 10 ${TTO:-700} python -u -m pytest $T -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 700 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r5/bench_summary.py $O/bench.json > $O/summary.txt; cat $O/summary.txt
