#!/bin/bash
# kernel names + average durations of hipBLASLt on the step's GEMM shapes (tools/calib_blas.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/blasnames; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/calib_blas.py > $O/out.jsonl 2> $O/err.log || { tail $O/err.log; exit 1; }
find $O -name '*kernel_trace.csv' -delete
python3 - <<PY
import csv, glob
f = glob.glob("$O/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:20]:
    print(f'{int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.1f}us  {r["Name"][:200]}')
PY
