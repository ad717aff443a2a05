#!/bin/bash
# two-half wgrad workgroups: op tests, the whole GPU suite with MTTS_WGRAD_HV=2, then a same-box step A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/hv; mkdir -p $O; cd $R
MTTS_WGRAD_HV=2 timeout -k 10 300 python -u -m pytest tests/test_decoder_ops_gpu.py -x -q -k wgrad --timeout 120 --timeout-method thread > $O/ops.log 2>&1; rc=$?
echo "wgrad ops rc=$rc"; tail -3 $O/ops.log; [ $rc -ne 0 ] && exit $rc
MTTS_WGRAD_HV=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/all.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|^FAILED" $O/all.log | tail -4; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab3.sh DUMMY=0 MTTS_WGRAD_HV=2 MTTS_WGRAD_HV=2,MTTS_WGRAD_MINBLK16=768,MTTS_WGRAD_MINBLK=512 DUMMY=0 MTTS_WGRAD_HV=2 MTTS_WGRAD_HV=2,MTTS_WGRAD_MINBLK16=768,MTTS_WGRAD_MINBLK=512
