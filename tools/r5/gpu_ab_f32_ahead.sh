#!/bin/bash
# round 5: exact-fp32 register schedules with every fragment of a K step read ahead of its MFMAs
# (MTTS_F32_FRAG_AHEAD; the noahead build: MTTS_BUILD_VARIANT=noahead MTTS_EXTRA_HIPCC_FLAGS=-DMTTS_F32_FRAG_AHEAD=0): GEMM tests,
# the step A/B alternating on one box -> gpurun_out/$TAG.  The read-ahead variant was measured slower and removed
#  without being committed: re-apply it (the fp32 branch of compute() reading all 16 fragment
# pairs, then a sched_barrier, the 16 MFMAs, another sched_barrier) to rerun this A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r5ahead}; mkdir -p $O; cd $R
NOAHEAD=matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip_noahead.so
PIN=matcha-tts-etu-upmc-ensam_amd/lib/libmtts_hip.so
timeout -k 10 400 python -u -m pytest tests/test_gemm_wreg_gpu.py tests/test_decoder_ops_gpu.py tests/test_encoder_ops_gpu.py tests/test_weight_split_gpu.py tests/test_headline_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for L in $NOAHEAD $PIN; do
  n=$(basename $L .so)
  MTTS_LIB=$L timeout -k 10 300 python -u tools/r5/gemm_replay.py profiles/r05/gemm_log_parity.jsonl --cfgs=-1 --out $O/replay_$n.jsonl > $O/replay_$n.log 2>&1 || { echo "replay $n failed"; tail -5 $O/replay_$n.log; exit 1; }
  tail -1 $O/replay_$n.log
done
VAR=MTTS_LIB A=$NOAHEAD B=$PIN TAG=${TAG:-r5ahead} bash tools/r5/gpu_ab_env.sh
