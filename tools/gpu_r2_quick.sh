#!/bin/bash
# quick loop: selected GPU tests + default bench (no CPU baseline)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r2q}; O=gpurun_out/$TAG; mkdir -p $O; shift
TESTS=${TESTS:-"tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_training_gpu.py"}
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E  |FAILED" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth "$@" > $O/bench.json 2> $O/bench.err; rc=$?
[ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python - <<PY
import json
d=json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "prec", d["precision_check"])
for k in ("roofline","roofline_wgrad","roofline_attn"):
    r=d[k]; print(k, r["bound"], r["achieved"], r["unit"], "frac", r["frac"], "avg_us", r["avg_launch_us"], "n", r["launches_per_step"], "TF", r["mfma_tflops"])
PY
