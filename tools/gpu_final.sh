#!/bin/bash
# Round artifacts on the GPU box: GPU tests, smoke, the default bench line (with CPU baseline), and a
# rocprofv3 kernel-trace summary of the same bench command.  Usage: bash tools/gpu_final.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; TAG=${1:-final}; mkdir -p $O/$TAG; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/$TAG/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|^FAILED" $O/$TAG/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/$TAG/smoke.log 2>&1; rc=$?
tail -2 $O/$TAG/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $O/$TAG/bench.json 2> $O/$TAG/bench.err; rc=$?; tail -c 2500 $O/$TAG/bench.json; [ $rc -ne 0 ] && { tail -20 $O/$TAG/bench.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/$TAG/prof_bench.json 2> $O/$TAG/prof.err; rc=$?
echo "prof rc=$rc"; exit $rc
