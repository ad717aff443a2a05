#!/bin/bash
# (ran on the tail-split experiment of round 6, since reverted: profiles/r06/tail_split/)
# tail split of the LDS-DMA GEMMs: its tests, replay of the step's bf16 launches with the split off / on, a timeline,
# bench A/B (alternating), then the whole GPU suite -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6tail}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm_tail_gpu.py -q -x --timeout 120 --timeout-method thread > $O/tail_tests.log 2>&1; rc=$?
tail -3 $O/tail_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/tail_tests.log | head -20; exit $rc; }
for t in 0 1; do
  MTTS_GEMM_TAIL=$t timeout -k 10 400 python -u tools/r5/gemm_replay.py profiles/r05/gemm_log_parity.jsonl --only-bf16 --cfgs=-1 --out $O/replay_tail$t.jsonl > $O/replay_tail$t.log 2>&1 || { echo "replay rc=$?"; tail -5 $O/replay_tail$t.log; exit 1; }
  tail -1 $O/replay_tail$t.log
done
timeout -k 10 120 python3 -u tools/r6/glds_timeline.py --match 9600,256,768,3,79 --out $O/tl_9600_79.json > $O/tl.log 2>&1 || { tail -5 $O/tl.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/tl_9600_79.json')); print('timeline (tail on)', {k: d[k] for k in ('kernel_us','wave_life_us_mean','waves','start_quantiles_us')})"
for i in 1 2; do
  for t in 0 1; do
    MTTS_GEMM_TAIL=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 30 > $O/bench_tail$t.$i.json 2> $O/bench_tail$t.$i.err || { echo "bench rc=$?"; tail -5 $O/bench_tail$t.$i.err; exit 1; }
    python -c "import json,sys; s=open(sys.argv[1]).read(); d=json.loads(s[s.index('{'):]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], d['precision_check']['bf16_loss_rel_err'], d['roofline']['avg_launch_us'])" $O/bench_tail$t.$i.json
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
exit 0
