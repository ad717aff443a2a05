#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -m pytest tests/test_decoder_ops_gpu.py -q > $O/ops_tests.log 2>&1; rc=$?; echo "ops rc=$rc"; grep -E "passed|failed|Error" $O/ops_tests.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -m pytest tests -m gpu -q -x --deselect tests/test_decoder_ops_gpu.py > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_f32.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench_f32.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --precision bf16-mixed --no-cpu-baseline > $O/bench_bf16.log 2>&1; rc=$?; echo "bench bf16 rc=$rc"; tail -c 600 $O/bench_bf16.log
