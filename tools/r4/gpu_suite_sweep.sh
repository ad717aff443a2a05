#!/bin/bash
# round 4: GPU suite, then the split-weight (bf16-parity) step GEMM sweep on the decoder-sized calls, then the bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4sw}; mkdir -p $O; cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -q --maxfail 6 --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .{0,200}" $O/gpu_tests.log | head -20; }
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
SWEEP_PREC=bf16-parity SWEEP_MIN_ROWS=9600 SWEEP_SPLITS=1 SWEEP_GLDS=32-47 timeout -k 10 600 python tools/r3/gemm_step_sweep.py > $O/ws_sweep.jsonl 2> $O/ws_sweep.err || { tail -5 $O/ws_sweep.err; exit 1; }
wc -l $O/ws_sweep.jsonl
timeout -k 10 400 python bench.py --no-extra --no-cpu-baseline > $O/bench.json 2> $O/bench.err && python tools/r4/bench_summary.py $O/bench.json
exit $rc
