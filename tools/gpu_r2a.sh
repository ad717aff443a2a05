#!/bin/bash
# round 2, first box: packed-fp32 fault probe + reproduction, full GPU suite, bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 120 tools/bin/pkprobe 4000 > $O/pkprobe.log 2>&1 || { echo probe failed; cat $O/pkprobe.log; exit 1; }
cat $O/pkprobe.log
MTTS_LIB=$R/matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_pk.so timeout -k 10 240 python -u tools/wgrad_debug.py > $O/wgrad_pk.log 2>&1 || { echo wgrad_debug failed; tail -20 $O/wgrad_pk.log; exit 1; }
tail -12 $O/wgrad_pk.log
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench_err.txt || { tail -20 $O/bench_err.txt; exit 1; }
cat $O/bench.json
