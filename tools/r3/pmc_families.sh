#!/bin/bash
# HBM traffic per launch of the step's three kernel families, as MI355X_MICROARCH.md's HBM/rocprofv3
# section prescribes: FETCH_SIZE and WRITE_SIZE in separate --pmc passes (they do not fit one TCC pass),
# per family (--kernel-include-regex), FETCH_SIZE doubled on gfx950.  -> gpurun_out/$TAG, profiles/$PROF
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-pmc3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for fam in gemm wgrad attn; do
  rx=$(python3 -c "import sys; sys.path.insert(0, '$R/tools/r3'); from pmc_regex import REGEX; print(REGEX['$fam'])")
  for c in FETCH_SIZE WRITE_SIZE; do
    sub=$([ $c = FETCH_SIZE ] && echo fetch || echo write)
    timeout -k 10 200 rocprofv3 --pmc $c --kernel-include-regex "$rx" --output-format csv -d $O/${fam}_$sub -o run -- python3 $R/tools/r3/pmc_families.py $O/algo.json > $O/${fam}_$sub.log 2>&1; rc=$?
    echo "$fam $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/${fam}_$sub.log; exit $rc; }
  done
done
cd $R/tools/r3 && python3 pmc_families_summary.py $O $R/gpurun_out/${TAG:-pmc3}/profiles
