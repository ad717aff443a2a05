#!/bin/bash
# per-wave timelines of the step's LDS-DMA GEMM launches (diagnostic lib/libmtts_hip_tl.so) -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6gtl}; mkdir -p $O; cd $R
for m in 9600,256,768,3,77 9600,256,768,3,79 19200,256,768,3,79 9600,256,1024,1,74 9600,256,768,3,10 9600,256,256,1,74 19200,256,1024,1,74; do
  timeout -k 10 120 python3 -u tools/r6/glds_timeline.py --match $m --out $O/tl_${m//,/_}.json > $O/tl_${m//,/_}.log 2>&1 || { echo "fail $m"; tail -5 $O/tl_${m//,/_}.log; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['shape'], 'ev %.1f kern %.1f life %.1f start90 %.1f pro %.2f first_wait %.2f loop %.1f epi %.2f wait %.2f comp %.2f steps %d waves %d w/cu %d-%d' % (d['event_us'], d['kernel_us'], d['wave_life_us_mean'], d['start_quantiles_us'][2], d['prologue_issue_us_mean'], d['first_wait_us_mean'], d['loop_us_mean'], d['epilogue_us_mean'], d['per_step_wait_us_mean'] or 0, d['per_step_compute_us_mean'], d['steps_recorded'], d['waves'], d['waves_per_cu_min'], d['waves_per_cu_max']))" $O/tl_${m//,/_}.json
done
