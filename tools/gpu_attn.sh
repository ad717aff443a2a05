#!/bin/bash
# attention GPU tests, one bench line, then a kernel-trace profile of the bench -> gpurun_out/$1/
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-attn}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|^FAILED|Error" $O/tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 30 > $O/bench.json 2>$O/bench.err || exit 1
python -c "import json;r=json.load(open('$O/bench.json'));print(r['value'], r['ms_per_step'])"
bash tools/gpu_prof_bench.sh ${1:-attn}
