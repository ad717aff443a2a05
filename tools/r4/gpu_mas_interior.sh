#!/bin/bash
# round 4: interior-chunk fast path of both DP kernels -- MAS / long-form / headline tests, maximum_path and
# fused-alignment timing (row-major and transposed), then one bench line -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4int}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_mas_gpu.py tests/test_longform_gpu.py tests/test_headline_gpu.py tests/test_native_abi.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|^E  " $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for TR in auto 0 1; do
  if [ $TR = auto ]; then unset MTTS_MAS_TR; else export MTTS_MAS_TR=$TR; fi
  timeout -k 10 200 python tools/mas_bench.py --configs 32x120x600,8x256x2048,8x512x4096,8x1024x4096,8x2048x4096 --iters 30 > $O/mas_$TR.jsonl 2>/dev/null || exit $?
  timeout -k 10 200 python tools/prior_mas_bench.py --configs 32x120x600,8x512x4096,8x1024x4096 --iters 30 > $O/prior_$TR.jsonl 2>/dev/null || exit $?
  echo "TR=$TR"; cat $O/mas_$TR.jsonl $O/prior_$TR.jsonl
done
unset MTTS_MAS_TR
timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/bench.json 2>/dev/null || exit $?
python tools/r4/bench_summary.py $O/bench.json | head -3
