#!/bin/bash
# Round-end artifacts in one call: PMC HBM traffic of the GEMM launches (-> profiles/r01/conv_gemm_traffic.json
# on the box, read by the bench), then tests + smoke + bench + rocprof summary (tools/gpu_final.sh TAG).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-final}
bash tools/pmc_traffic.sh pmc_$TAG || exit $?
python tools/pmc_summary.py gpurun_out/pmc_$TAG gpurun_out/pmc_$TAG/conv_gemm_traffic.json || exit $?
cp gpurun_out/pmc_$TAG/conv_gemm_traffic.json profiles/r01/conv_gemm_traffic.json
bash tools/gpu_final.sh $TAG
