#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r2d; mkdir -p $O
echo "== E: current source, packed-fp32 build, generic (INC=false) wgrad"
MTTS_LIB=$R/matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_pk.so timeout -k 10 200 python -u tools/wgrad_generic_check.py > $O/E.log 2>&1; echo "rc $?"; cat $O/E.log | grep -v amdgpu.ids
echo "== E0: current source, product build, generic wgrad"
timeout -k 10 200 python -u tools/wgrad_generic_check.py > $O/E0.log 2>&1; echo "rc $?"; grep -v amdgpu.ids $O/E0.log
echo "== F: 323f289 + select for the dY mask, packed-fp32 build"
(cd tools/bin/w323F && timeout -k 10 200 python -u tools/wgrad_debug.py > $O/F.log 2>&1) || { echo F failed; tail $O/F.log; exit 1; }
grep -c "bad 0 " $O/F.log; grep -v "bad 0 " $O/F.log | head -4
