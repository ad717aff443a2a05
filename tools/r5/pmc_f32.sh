set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r5pmc_f32/up MATCH="3840,768,576,1,3" CFGS="-1,18" bash tools/r5/pmc_gemm.sh && \
TAG=r5pmc_f32/down MATCH="3840,192,2304,0,0" CFGS="-1,18" bash tools/r5/pmc_gemm.sh && \
timeout -k 10 120 python3 -u tools/r5/gemm_replay.py profiles/r05/gemm_log_parity.jsonl --match "3840,768,576,1,3" --cfgs=-1,18,3,11,7 > gpurun_out/r5pmc_f32/replay_up.log 2>&1
