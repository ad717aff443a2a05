mkdir -p gpurun_out/r5tl && \
timeout -k 10 120 python3 -u tools/r5/gemm_timeline.py --match 3840,768,576,1,3 --out gpurun_out/r5tl/ffn_up.json > gpurun_out/r5tl/ffn_up.log 2>&1 && \
timeout -k 10 120 python3 -u tools/r5/gemm_timeline.py --match 3840,192,2304,0,0 --out gpurun_out/r5tl/ffn_down.json > gpurun_out/r5tl/ffn_down.log 2>&1 && \
timeout -k 10 120 python3 -u tools/r5/gemm_timeline.py --match 3840,576,192,1,0 --out gpurun_out/r5tl/qkv.json > gpurun_out/r5tl/qkv.log 2>&1
