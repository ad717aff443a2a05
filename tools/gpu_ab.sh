#!/bin/bash
# A/B of an env switch: bench + rocprofv3 kernel stats for each setting.  Usage: gpu_ab.sh TAG VAR VAL_A VAL_B
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; VAR=$2; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in $3 $4; do
  export $VAR=$v
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-synth --steps 40 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]);print('$VAR=$v', d['value'], d['ms_per_step'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 $R/bench.py --no-cpu-baseline --no-synth --steps 20 --warmup 3 > $O/prof_$v.out 2> $O/prof_$v.err || { tail -20 $O/prof_$v.err; exit 1; }
  find $O/prof_$v -name '*kernel_trace.csv' -delete
done
for v in $3 $4; do echo "== $VAR=$v"; python3 $R/tools/kstats.py $(find $O/prof_$v -name '*kernel_stats.csv' | head -1) 20 18; done
