set -e
mkdir -p gpurun_out
export PRA_TUNE_MS=40 PRA_TUNE_ITERS=20
timeout -k 10 600 python tools/gemm_bench.py --layouts --only w2,wo --tune gpurun_out/tune_w2.csv > gpurun_out/gemm_w2_tune.log 2>&1
tail -1 gpurun_out/gemm_w2_tune.log
