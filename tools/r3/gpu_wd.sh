#!/bin/bash
# batched wgrads flushed at the end (inline 0): split-count sweep (same box) + profile
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3wd}; mkdir -p $O; cd $R
export MTTS_INLINE_REDUCE_JOBS=0
for rep in 1 2; do for cfg in "384 512 768" "256 256 768" "128 128 768" "128 128 1536" "64 64 3072" "256 256 1536"; do set -- $cfg
  MTTS_WGRAD_MINBLK=$1 MTTS_WGRAD_MINBLK16=$2 MTTS_WGRAD_ROWS=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/ab.json 2> $O/ab.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/ab.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/ab.json')); print('minblk=$1/$2 rows=$3 rep $rep', d['ms_per_step'])"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/prof.err; exit $rc; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $T $O/trace.csv
python3 $R/tools/step_breakdown.py $T > $O/step.txt; head -14 $O/step.txt
python3 $R/tools/r3/step_phases.py $T | tee $O/phases.txt
