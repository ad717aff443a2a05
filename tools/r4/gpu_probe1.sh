#!/bin/bash
# round 4: MAS one-wave vs multi-wave A/B (tools/mas_bench.py), the FFN up-projection probe
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4p1}; mkdir -p $O; cd $R
for MW in 0 1; do
  MTTS_MAS_MW=$MW timeout -k 10 200 python tools/mas_bench.py --configs 32x120x600,8x512x4096,8x256x2048 > $O/mas_mw$MW.jsonl 2>&1 || { tail -3 $O/mas_mw$MW.jsonl; exit 1; }
  echo "mw=$MW"; cat $O/mas_mw$MW.jsonl
done
timeout -k 10 400 python tools/r4/ff1_probe.py > $O/ff1_probe.txt 2>&1 || { tail -3 $O/ff1_probe.txt; exit 1; }
cat $O/ff1_probe.txt
