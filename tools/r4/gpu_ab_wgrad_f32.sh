#!/bin/bash
# round 4: fp32 encoder-forward GEMM sweep; in-kernel wgrad sums (protocol 2) tests + same-box bench A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4ab}; mkdir -p $O; cd $R
timeout -k 10 400 python tools/r4/gemm_f32_sweep.py > $O/f32_sweep.jsonl 2> $O/f32_sweep.err || { tail -5 $O/f32_sweep.err; exit 1; }
tail -1 $O/f32_sweep.jsonl
MTTS_WGRAD_FUSED_SUM=2 timeout -k 10 300 python -u -m pytest tests/test_training_gpu.py tests/test_decoder_ops_gpu.py tests/test_dp_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/proto2_tests.log 2>&1; rc=$?
tail -2 $O/proto2_tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .{0,200}" $O/proto2_tests.log | head -10; }
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
for i in 1 2; do
  for F in 0 2; do
    MTTS_WGRAD_FUSED_SUM=$F timeout -k 10 200 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/bench_f$F.$i.json 2>/dev/null || exit $?
    echo "fused=$F run $i: $(python -c "import json,sys; d=json.loads([l for l in open('$O/bench_f$F.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'])")"
  done
done
