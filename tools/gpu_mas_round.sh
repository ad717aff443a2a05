#!/bin/bash
# First GPU pass: MAS parity tests, timing, rocprof kernel trace. Stops on any fault/timeout.
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
mkdir -p $R/gpurun_out
timeout -k 10 400 python -m pytest $R/tests/test_mas_gpu.py -x -q > $R/gpurun_out/mas_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -5 $R/gpurun_out/mas_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python $R/tools/mas_bench.py --cpu > $R/gpurun_out/mas_bench.log 2>&1 || { echo bench_fail; cat $R/gpurun_out/mas_bench.log | tail; exit 3; }
cat $R/gpurun_out/mas_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_mas -o mas -- python3 $R/tools/mas_bench.py --iters 20 > $R/gpurun_out/prof_mas.log 2>&1
echo "prof_rc=$?"
find $R/gpurun_out/prof_mas -name "*stats*" | head
