#!/bin/bash
# LDS-DMA GEMM schedules: epilogue equivalence + timing sweep vs the register-staged default (cfg 12).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python tools/gemm_sweep.py bf16 ${1:-12,32,33,34,35,36,37,38,39,40,41,42,43} > $O/glds_sweep.log 2>&1; rc=$?
grep -v amdgpu.ids $O/glds_sweep.log | tail -250; exit $rc
