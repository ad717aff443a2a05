#!/bin/bash
# packed-fp32 fault: operand-select probe + round-1 wgrad builds with packed fp32 re-enabled
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r2b; mkdir -p $O
timeout -k 10 150 tools/bin/pkprobe 4000 > $O/pkprobe.log 2>&1 || { echo probe failed; cat $O/pkprobe.log; exit 1; }
cat $O/pkprobe.log
for c in 323f289 ab14996; do
  (cd tools/bin/w$c && timeout -k 10 200 python -u tools/wgrad_debug.py > $O/wgrad_w$c.log 2>&1) || { echo wgrad $c failed; tail -20 $O/wgrad_w$c.log; exit 1; }
  echo "== $c"; grep -c "bad 0 " $O/wgrad_w$c.log; grep -v "bad 0 " $O/wgrad_w$c.log | head -8
done
MTTS_LIB=$R/matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_pk.so timeout -k 10 300 python -u -m pytest tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pk_tests.txt 2>&1; echo "pk tests rc $?"; tail -3 $O/pk_tests.txt
