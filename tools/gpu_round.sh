#!/bin/bash
# One GPU session: smoke, GPU tests, bench (fp32 + bf16), rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script there.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
stop() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc at $2"; exit $rc; fi; }
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; stop $rc smoke
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/gpu_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log; stop $rc tests
timeout -k 10 400 python bench.py > $O/bench_f32.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_f32.log; stop $rc bench
timeout -k 10 300 python bench.py --precision bf16-mixed --no-cpu-baseline > $O/bench_bf16.log 2>&1; rc=$?; echo "bench bf16 rc=$rc"; tail -1 $O/bench_bf16.log; stop $rc bench_bf16
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1; rc=$?; echo "prof rc=$rc"; stop $rc prof
find $O/prof_bench -name "*stats*"
