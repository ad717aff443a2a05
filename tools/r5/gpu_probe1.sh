#!/bin/bash
# round 5 first probe: L2->LDS fill rates (tools/r5/fill_probe.hip) + the default bench step's GEMM launch list
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5p1}; mkdir -p $O; cd $R
timeout -k 10 120 ./tools/bin/fill_probe > $O/fill.jsonl 2> $O/fill.err || { echo "fill rc=$?"; tail -5 $O/fill.err; exit 1; }
echo fill-done; wc -l $O/fill.jsonl
MTTS_DUMP_GEMM_LOG=$O/gemm_log.jsonl timeout -k 10 400 python bench.py --no-extra --no-cpu-baseline --no-synth --no-graph-profile > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python tools/r4/bench_summary.py $O/bench.json | head -5; wc -l $O/gemm_log.jsonl
