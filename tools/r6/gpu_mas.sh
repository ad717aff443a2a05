#!/bin/bash
# multi-wave MAS DP (round 6: per-column issue trimmed): bit-exact MAS tests, maximum_path timing vs the CPU oracle
# (bit_exact), and the long-form config-5 bench line (roofline_mas.chain_bound) -> gpurun_out/$TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-r6mas}; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_mas_gpu.py tests/test_longform_gpu.py -q -x --timeout 300 --timeout-method thread > $O/mas_tests.log 2>&1; rc=$?
tail -3 $O/mas_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" $O/mas_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/mas_bench.py --iters 30 --cpu --configs 32x120x600,8x256x2048,8x512x4096,8x1024x4096 > $O/mas_bench.jsonl 2> $O/mas_bench.err || { tail -5 $O/mas_bench.err; exit 1; }
cat $O/mas_bench.jsonl
timeout -k 10 400 python bench.py --batch 8 --tx 512 --ty 4096 --no-extra --no-cpu-baseline --no-synth > $O/longform_max.json 2> $O/lf1.err || { tail -5 $O/lf1.err; exit 1; }
python -c "import json,sys; s=open(sys.argv[1]).read(); d=json.loads(s[s.index('{'):]); print('longform ms', d['ms_per_step'], json.dumps(d['roofline_mas']['chain_bound']), d['graph_replay_profile']['top_kernels_us'].get('mas_dp_mw_kernel'))" $O/longform_max.json
