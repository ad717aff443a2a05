#!/bin/bash
# A/B of two builds in one box: the committed-before build copied to lib/ab/ vs the current lib/,
# bench alternated twice (no CPU baseline); optional TESTS run first on the current build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-libab}; O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1; rc=$?
  tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "^E  |FAILED" $O/tests.log | head -20; exit $rc; }
fi
for i in 1 2; do
  for L in ab cur; do
    # AB_ENV: settings the baseline leg needs (e.g. switching off a feature the older build lacks)
    if [ $L = ab ]; then export MTTS_LIB=$R/matcha-tts-etu-upmc-ensam_amd/lib/ab/libmtts_hip.so; for kv in $AB_ENV; do export $kv; done
    else unset MTTS_LIB; for kv in $AB_ENV; do unset ${kv%%=*}; done; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-synth --steps 40 > $O/b_${L}_$i.json 2> $O/b_${L}_$i.err || { tail -5 $O/b_${L}_$i.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${L}_$i.json').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
