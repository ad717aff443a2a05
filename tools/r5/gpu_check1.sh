#!/bin/bash
# round 5: parity + training tests touched this round, a full bench line with extras, the pk replay
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5c1}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_training_gpu.py tests/test_decoder_ops_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -s > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "grad|FAILED" $O/tests.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r5/bench_summary.py $O/bench.json | head -16
TAG=${TAG:-r5c1}/rp ARGS="--top 12" CFGS=-1,44,77,78,79,80 TO=300 bash tools/r5/gpu_replay.sh
