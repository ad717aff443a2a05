#!/bin/bash
# op tests + bench (both precisions) + profile of bf16 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -m pytest tests/test_decoder_ops_gpu.py tests/test_model_gpu.py -q > $O/ops_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error" $O/ops_tests.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for P in 32-true bf16-mixed; do
timeout -k 10 300 python bench.py --no-cpu-baseline --precision $P > $O/bench_$P.log 2>&1; rc=$?; echo "bench $P rc=$rc"; python -c "import json,sys; d=json.loads(open('$O/bench_$P.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['maximum_path']['ms_per_call'])"
if [ $rc -ne 0 ]; then exit $rc; fi
done
bash $R/tools/gpu_prof.sh prof_bf16 --precision bf16-mixed --steps 10 --warmup 3 > /dev/null 2>&1; echo prof rc=$?
