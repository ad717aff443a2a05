#!/bin/bash
# round 4: the DP on the transposed lattice -- MAS tests, maximum_path timing with MTTS_MAS_TR=1 / 0, SQ counters
# of the transposed DP at 8x512x4096, then the bench line + parity-step profile -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4tr}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_mas_gpu.py tests/test_longform_gpu.py tests/test_headline_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|^E  " $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for TR in 1 0; do
  MTTS_MAS_TR=$TR timeout -k 10 200 python tools/mas_bench.py --configs 8x512x4096,32x120x600,8x256x2048,8x1024x4096 --iters 30 > $O/mas_tr$TR.jsonl 2>/dev/null || exit $?
  echo "TR=$TR"; cat $O/mas_tr$TR.jsonl
done
timeout -k 10 600 bash tools/pmc_sq.sh mas_dp tools/r4/mas_pmc_run.py 8x512x4096 || exit $?
python tools/pmc_sq_summary.py gpurun_out/pmc_sq > $O/mas_pmc.txt 2>&1; grep -E "mas_dp|WAVE_CYCLES|WAIT_ANY|WAIT_INST_ANY|ACTIVE_INST_ANY|INSTS_VALU" $O/mas_pmc.txt
rm -rf $O/pmc_sq; mv gpurun_out/pmc_sq $O/pmc_sq
TAG=${TAG:-r4tr}/b SUITE=0 SMOKE=0 BENCH=1 BENCH_ARGS="--no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30" bash tools/r4/gpu_bench_prof.sh
