#!/bin/bash
# (ran on the weight-resident schedule of round 6, since removed: profiles/r06/wlds/)
# weight-resident GEMM (csrc/conv_gemm_wlds.hip): its tests, a replay of the step's bf16 GEMM launches on the
# heuristic vs the new schedule, and bench A/B with the heuristic pick off / on -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6wlds}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm_wlds_gpu.py tests/test_gemm_wreg_gpu.py -q -x --timeout 120 --timeout-method thread > $O/wlds_tests.log 2>&1; rc=$?
tail -3 $O/wlds_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/wlds_tests.log | head -20; exit $rc; }
timeout -k 10 400 python -u tools/r5/gemm_replay.py profiles/r05/gemm_log_parity.jsonl --only-bf16 --cfgs=-1,64 --out $O/replay.jsonl > $O/replay.log 2>&1; rc=$?
tail -5 $O/replay.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for pick in 0 1; do
    MTTS_GEMM_WLDS_PICK=$pick timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 30 > $O/bench_pick$pick.$i.json 2> $O/bench_pick$pick.$i.err || { echo "bench rc=$?"; tail -5 $O/bench_pick$pick.$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['precision_check']['bf16_loss_rel_err'])" $O/bench_pick$pick.$i.json
  done
done
