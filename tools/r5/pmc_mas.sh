#!/bin/bash
# HBM traffic of maximum_path on the bench lattice (FETCH_SIZE / WRITE_SIZE in separate --pmc passes, the
# mas_* kernels only) -> gpurun_out/$TAG/profiles/mas_traffic_parity.json (bench.py roofline_mas.traffic)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5pmcmas}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  sub=$([ $c = FETCH_SIZE ] && echo fetch || echo write)
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "mas_" --output-format csv -d $O/mas_$sub -o run -- python3 $R/tools/r5/pmc_mas.py $O/algo.json > $O/mas_$sub.log 2>&1; rc=$?
  echo "mas $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/mas_$sub.log; exit $rc; }
done
cd $R/tools/r3 && python3 pmc_families_summary.py $O $O/profiles mas
