#!/bin/bash
# round 5: the register-staged GEMM / weight-gradient loops with and without the prefetch scheduling fence
# (MTTS_PIN_PREFETCH): GEMM tests on the fenced build, replay of the step's GEMM launches on both builds, then
# the step A/B alternating on one box -> gpurun_out/$TAG.  The unfenced build, beside the default one:
#   MTTS_BUILD_VARIANT=nopin MTTS_EXTRA_HIPCC_FLAGS=-DMTTS_PIN_PREFETCH=0 python matcha-tts-etu-upmc-ensam_amd/build_native.py
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5pin}; mkdir -p $O; cd $R
NOPIN=matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_nopin.so
PIN=matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gemm_wreg_gpu.py tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_weight_split_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for L in $NOPIN $PIN; do
  n=$(basename $L .so)
  MTTS_LIB=$L timeout -k 10 300 python -u tools/r5/gemm_replay.py profiles/r05/gemm_log_parity.jsonl --cfgs=-1 --out $O/replay_$n.jsonl > $O/replay_$n.log 2>&1 || { echo "replay $n failed"; tail -5 $O/replay_$n.log; exit 1; }
  tail -1 $O/replay_$n.log
done
VAR=MTTS_LIB A=$NOPIN B=$PIN TAG=${TAG:-r5pin} bash tools/r5/gpu_ab_env.sh
