#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r2f; mkdir -p $O
PK=$R/matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_pk.so
echo "== E': select fix, packed-fp32 build, generic wgrad"
MTTS_LIB=$PK timeout -k 10 200 python -u tools/wgrad_generic_check.py > $O/E2.log 2>&1; echo "rc $?"; grep -v amdgpu.ids $O/E2.log
echo "== wgrad/gemm exactness, product build"
timeout -k 10 300 python -u -m pytest tests/test_decoder_ops_gpu.py -k "exact_and_deterministic" -m gpu -x -q --timeout 120 --timeout-method thread > $O/exact.txt 2>&1; echo "rc $?"; tail -2 $O/exact.txt
echo "== all op tests, packed-fp32 build"
MTTS_LIB=$PK timeout -k 10 300 python -u -m pytest tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pk_ops.txt 2>&1; echo "rc $?"; tail -2 $O/pk_ops.txt
