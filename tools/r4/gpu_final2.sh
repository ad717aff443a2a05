#!/bin/bash
# round 4, second final snapshot on HEAD: prefetch A/B (MTTS_PREFETCH=1 / 0), then the default bench line with
# extras, the parity-step rocprofv3 profile and the long-form lines (PMC passes unchanged: PMC=0) -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4final2}; mkdir -p $O; cd $R
for i in 1 2; do
  for P in 1 0; do
    MTTS_PREFETCH=$P timeout -k 10 300 python bench.py --no-extra --no-graph-profile --no-synth --no-cpu-baseline --steps 30 > $O/ab_prefetch$P.$i.json 2>/dev/null || exit $?
    echo "prefetch=$P run $i: $(python -c "import json; d=json.loads([l for l in open('$O/ab_prefetch$P.$i.json') if l.startswith('{')][-1]); print(d['ms_per_step'])")"
  done
done
TAG=${TAG:-r4final2} SUITE=0 SMOKE=0 BENCH=1 bash tools/r4/gpu_suite.sh || exit $?
TAG=${TAG:-r4final2}/prof PREC=bf16-parity bash tools/r4/gpu_prof.sh || exit $?
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --no-extra --no-cpu-baseline --no-synth > $O/longform_max.json 2> $O/lf1.err || { tail -5 $O/lf1.err; exit 1; }
python tools/r4/bench_summary.py $O/longform_max.json | head -2
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --bucketed 4 --no-extra --no-cpu-baseline --no-synth --no-graph-profile > $O/longform_bucketed.json 2> $O/lf2.err || { tail -5 $O/lf2.err; exit 1; }
python tools/r4/bench_summary.py $O/longform_bucketed.json | head -2
echo final2-done
