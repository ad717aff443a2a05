#!/bin/bash
# A/B of the forced-DP step (world 1) against the plain step, alternating, on one box: plain, DP (optimizer
# inside the fwd/bwd graph), DP with MTTS_DP_SPLIT_OPT=1 -> gpurun_out/$TAG/ab.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5abdp}; mkdir -p $O; cd $R
A="--no-extra --no-synth --no-cpu-baseline --no-graph-profile --steps 40 --warmup 5"
timeout -k 10 200 python -u -m pytest tests/test_dp_gpu.py -q -x --timeout 120 --timeout-method thread > $O/t0.log 2>&1 || { tail -5 $O/t0.log; exit 1; }
MTTS_DP_SPLIT_OPT=1 timeout -k 10 200 python -u -m pytest tests/test_dp_gpu.py -q -x --timeout 120 --timeout-method thread > $O/t1.log 2>&1 || { tail -5 $O/t1.log; exit 1; }
tail -1 $O/t0.log $O/t1.log
: > $O/ab.txt
for rep in 1 2; do
  for v in plain dp dpsplit; do
    case $v in
      plain) E="" ;; dp) E="MTTS_FORCE_DP=1" ;; dpsplit) E="MTTS_FORCE_DP=1 MTTS_DP_SPLIT_OPT=1" ;;
    esac
    env $E timeout -k 10 300 python bench.py $A > $O/$v$rep.json 2> $O/$v$rep.err || { echo "$v failed"; tail -5 $O/$v$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/$v$rep.json').read().strip().splitlines()[-1]); print('$v', $rep, d['ms_per_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
