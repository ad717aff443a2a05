#!/bin/bash
# batched (deferred) weight gradients: tests, then same-box A/B of the defer switch and the inline-flush threshold
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wb}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_decoder_ops_gpu.py tests/test_dp_gpu.py tests/test_model_gpu.py tests/test_encoder_ops_gpu.py -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  " $O/tests.log | head -30; exit $rc; }
for rep in 1 2; do for cfg in "1 8" "0 8" "1 16" "1 32"; do set -- $cfg
  MTTS_DEFER_WGRAD=$1 MTTS_INLINE_REDUCE_JOBS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab_$1_$2_$rep.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab_$1_$2_$rep.json')); print('defer=$1 inline=$2 rep $rep', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $T $O/trace.csv
python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -12 $O/step.txt
python3 $R/tools/r3/step_phases.py $T | tee $O/phases.txt
