#!/bin/bash
# session-2 baseline: smoke, short bench, per-shape wgrad table, hipBLASLt wgrad calibration
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3w}; mkdir -p $O; cd $R
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '.'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log; [ $rc -ne 0 ] && { tail -20 $O/smoke.log; exit $rc; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'])"
timeout -k 10 200 python tools/step_wgrads.py > $O/wgrads.txt 2>&1; rc=$?; tail -30 $O/wgrads.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/calib_blas_wgrad.py > $O/calib_wgrad.txt 2>&1; rc=$?; cat $O/calib_wgrad.txt; exit $rc
