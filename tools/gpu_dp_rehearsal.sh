#!/bin/bash
# Two ranks on the one GPU over gloo: the graph-mode data-parallel step (captured fwd/bwd, one
# all-reduce of the flat gradient buffer, captured clip + AdamW) end to end, plus the eager DDP step.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
export MTTS_BENCH_SHARED_GPU=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 2 --batch 8 --no-synth > $O/dp_graph.log 2>&1; rc=$?
echo "graph rc=$rc"; grep '^{' $O/dp_graph.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['config']['parallelism'], d['losses'])" || tail -30 $O/dp_graph.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 2 --batch 8 --no-graph --no-synth > $O/dp_eager.log 2>&1; rc=$?
echo "eager rc=$rc"; grep '^{' $O/dp_eager.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d['losses'])" || tail -30 $O/dp_eager.log
exit $rc
