#!/bin/bash
# MAS GPU parity tests, then the fused alignment step + expand_rows_bwd timing (tools/prior_mas_bench.py).
# Usage: bash tools/gpu_mas_ring.sh [ring depths...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/mas_ring; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_mas_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for d in ${@:-4}; do
  MTTS_MAS_RING=$d timeout -k 10 120 python tools/prior_mas_bench.py >> $O/ring.jsonl 2>> $O/ring.err || exit $?
done
cat $O/ring.jsonl
