#!/bin/bash
# round 4: MAS tests + one-wave / multi-wave A/B, then the PMC traffic passes of the parity step -> profiles
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4pmc}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_mas_gpu.py -q --timeout 200 --timeout-method thread > $O/mas_tests.log 2>&1 || { tail -20 $O/mas_tests.log; exit 1; }
tail -1 $O/mas_tests.log
for MW in 0 1; do
  MTTS_MAS_MW=$MW timeout -k 10 200 python tools/mas_bench.py --configs 32x120x600,8x512x4096,8x256x2048 > $O/mas_mw$MW.jsonl 2>&1 || exit 1
  echo "mw=$MW"; grep config $O/mas_mw$MW.jsonl
done
PMC_PREC=bf16-parity TAG=${TAG:-r4pmc}/pmc bash tools/r3/pmc_families.sh
