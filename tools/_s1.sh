set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k attention --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
tail -2 gpurun_out/t_attn.log
timeout -k 10 120 python tools/attn_bench.py --B 8 > gpurun_out/attn_b8.log 2>&1
tail -1 gpurun_out/attn_b8.log
timeout -k 10 300 python tools/gemm_bench.py --layouts > gpurun_out/gemm_layouts.log 2>&1
tail -1 gpurun_out/gemm_layouts.log
