#!/bin/bash
# Data-path GPU checks: log-mel parity test, then the log-mel timing line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/data_path; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_data_path.py tests/test_mas_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/mel_bench.py > $O/mel_bench.json 2> $O/mel_bench.err; rc=$?; cat $O/mel_bench.json; exit $rc
