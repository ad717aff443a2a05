#!/bin/bash
# Round 3, first GPU pass: the whole -m gpu suite (incl. the 2-rank real-model DP test), the N=1 bench,
# `bench.py --gpus 2` self-spawning two ranks on the shared GPU (gloo), the bf16 error budget, the map of
# the step's torch kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3a}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
MTTS_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 3 --batch 8 --no-synth > $O/bench_shared2.json 2> $O/bench_shared2.err; rc=$?
echo "shared2 rc=$rc"; python -c "import json;d=json.loads(open('$O/bench_shared2.json').read().strip().splitlines()[-1]);print(d['n_gpus'],d['dp'],d['value'])" || tail -30 $O/bench_shared2.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/r3/precision_budget.py > $O/precision_budget.jsonl 2> $O/precision_budget.err; rc=$?
echo "budget rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/precision_budget.err; exit $rc; }
timeout -k 10 200 python tools/r3/glue_map.py $O/glue_map.txt > /dev/null 2> $O/glue_map.err; rc=$?
echo "glue rc=$rc"; head -3 $O/glue_map.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/r3/graph_event_probe.py > $O/graph_event_probe.txt 2>&1; rc=$?
cat $O/graph_event_probe.txt | grep -v amdgpu.ids; exit $rc
