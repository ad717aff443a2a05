#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r2c; mkdir -p $O
for c in 323A 323B; do
  (cd tools/bin/w$c && timeout -k 10 200 python -u tools/wgrad_debug.py > $O/wgrad_w$c.log 2>&1) || { echo wgrad $c failed; tail -20 $O/wgrad_w$c.log; exit 1; }
  echo "== $c"; grep -c "bad 0 " $O/wgrad_w$c.log; grep -v "bad 0 " $O/wgrad_w$c.log | head -4
done
