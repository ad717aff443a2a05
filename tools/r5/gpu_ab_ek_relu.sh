#!/bin/bash
# round 5: compile-time ReLU / ReLU' epilogue kinds (EK_RELU32 / EK_DRELU32) vs the run-time epilogue: GEMM / op
# tests on the default build, replay of the step's GEMM launches on both builds, the step A/B alternating on one box
# -> gpurun_out/$TAG.  The run-time build: MTTS_BUILD_VARIANT=rt MTTS_EXTRA_HIPCC_FLAGS=-DMTTS_EK_RELU=0
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5ekrelu}; mkdir -p $O; cd $R
RT=matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_rt.so
EK=matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gemm_wreg_gpu.py tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_weight_split_gpu.py tests/test_headline_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for L in $RT $EK; do
  n=$(basename $L .so)
  MTTS_LIB=$L timeout -k 10 300 python -u tools/r5/gemm_replay.py profiles/r05/gemm_log_parity.jsonl --cfgs=-1 --out $O/replay_$n.jsonl > $O/replay_$n.log 2>&1 || { echo "replay $n failed"; tail -5 $O/replay_$n.log; exit 1; }
  tail -1 $O/replay_$n.log
done
CONFIGS="MTTS_LIB=$RT;MTTS_LIB=$EK" REPS=3 TAG=${TAG:-r5ekrelu} bash tools/r5/gpu_ab_configs.sh
