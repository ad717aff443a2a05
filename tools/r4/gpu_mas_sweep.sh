#!/bin/bash
# round 4: DP shape sweep on the transposed lattice (MTTS_MAS_SHAPE = "W,KL", MTTS_MAS_TR_RING for the one-wave
# kernel): MAS tests first, then maximum_path (tools/mas_bench.py) and the fused training alignment
# (tools/prior_mas_bench.py) per shape -> gpurun_out/$TAG/sweep.jsonl
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r4sw2}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_mas_gpu.py tests/test_longform_gpu.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^FAILED|^E  " $O/tests.log | head -30; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CF=32x120x600,8x256x2048,8x512x4096,8x1024x4096
: > $O/sweep.jsonl
run() {  # $1 label; env already set by the caller
  timeout -k 10 200 python tools/mas_bench.py --configs $CF --iters 20 2>/dev/null | sed "s/^{/{\"shape\": \"$1\", \"tool\": \"maximum_path\", /" >> $O/sweep.jsonl || return 1
  timeout -k 10 200 python tools/prior_mas_bench.py --configs 32x120x600,8x512x4096,8x1024x4096 --iters 20 2>/dev/null | sed "s/^{/{\"shape\": \"$1\", \"tool\": \"prior\", /" >> $O/sweep.jsonl || return 1
}
MTTS_MAS_TR=0 run rowmajor || exit 1
run default || exit 1
for S in "1,0" "2,1" "2,2" "4,1" "4,2" "4,4" "8,1" "8,2" "8,4"; do MTTS_MAS_SHAPE=$S run "$S" || exit 1; done
for D in 2 8; do MTTS_MAS_SHAPE=1,0 MTTS_MAS_TR_RING=$D run "1,0-ring$D" || exit 1; done
python - $O/sweep.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
t = collections.defaultdict(dict)
for r in rows:
    key = (r["tool"], r.get("config") or r.get("cfg"))
    t[key][r["shape"]] = r.get("gpu_ms") or r.get("prior_maximum_path_ms")
for k, v in sorted(t.items()):
    print(k, " ".join(f"{s}:{ms}" for s, ms in v.items()))
PY
