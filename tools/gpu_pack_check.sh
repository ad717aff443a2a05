set -e
O=gpurun_out/pack32; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cfm_prep_gpu.py tests/test_model_gpu.py tests/test_training_gpu.py > $O/tests.txt 2>&1
tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-synth > $GRAFT_REPO_ROOT/$O/bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err
grep cfm_pack $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv | cut -c1-160
head -c 260 $GRAFT_REPO_ROOT/$O/bench.json
