set -e
O=gpurun_out/final_f; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
tail -3 $O/gpu_tests.txt
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -2 $O/smoke.txt
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench_err.txt
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
