#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_attention_gpu.py -x -q -m gpu > $O/attn_tests.log 2>&1; rc=$?; tail -25 $O/attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m pytest tests -q -m gpu -x > $O/gpu_tests.log 2>&1; rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_attn.json 2>&1; rc=$?; python -c "import json; d=json.loads(open('$O/bench_attn.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['losses'])"; exit $rc
