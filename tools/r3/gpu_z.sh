#!/bin/bash
# launch floor probe + bench under the kernel-argument placement switch
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r3z}; mkdir -p $O; cd $R
for v in unset 1 0; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 120 python tools/r3/launch_floor.py > $O/floor_$v.txt 2>&1; rc=$?; echo "== $v"; cat $O/floor_$v.txt | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-synth --no-extra --no-graph-profile --steps 20 --warmup 5 > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/bench_$v.err; exit $rc; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('bench', d['ms_per_step'])"
done
