#!/bin/bash
# BASELINE config 5 (long-form, B=8, Tx<=512, Ty<=4096) on one GPU, round 2: the synthetic max-length batch and
# 4 length-bucketed batches (bench.py --bucketed 4), each with a rocprofv3 kernel trace (alignment vs decoder).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/longform2; mkdir -p $O; cd $R
for mode in plain bucketed; do
  EXTRA=""; [ $mode = bucketed ] && EXTRA="--bucketed 4"
  ARGS="--batch 8 --tx 512 --ty 4096 --steps 12 --warmup 3 --no-cpu-baseline --no-synth $EXTRA"
  timeout -k 10 400 python bench.py $ARGS > $O/bench_$mode.json 2> $O/bench_$mode.err || { tail -20 $O/bench_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$mode.json').read().strip().splitlines()[-1]);print('$mode', d['value'], d['ms_per_step'])"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$mode -o run -- python3 $R/bench.py $ARGS > $O/prof_$mode.json 2> $O/prof_$mode.err) || { tail -5 $O/prof_$mode.err; exit 1; }
done
echo done
