#!/bin/bash
# round 4: optimizer tests, MAS long-form timing + SQ counter passes of the DP kernels, then the bench line and
# the parity-step profile -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4mas}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_training_gpu.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/mas_bench.py --configs 8x512x4096,32x120x600,8x256x2048 --iters 30 > $O/mas.jsonl 2>/dev/null || exit $?
cat $O/mas.jsonl
timeout -k 10 600 bash tools/pmc_sq.sh mas_dp tools/r4/mas_pmc_run.py 8x512x4096 || exit $?
python tools/pmc_sq_summary.py gpurun_out/pmc_sq > $O/mas_pmc.txt 2>&1; cat $O/mas_pmc.txt | head -40
rm -rf $O/pmc_sq; mv gpurun_out/pmc_sq $O/pmc_sq
TAG=${TAG:-r4mas}/b SUITE=0 SMOKE=0 BENCH=1 BENCH_ARGS="--no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30" bash tools/r4/gpu_bench_prof.sh
