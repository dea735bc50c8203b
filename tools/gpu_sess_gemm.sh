export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_nt_gpu.py tests/test_kernels_gpu.py -k "wgrad or gemm_nt or nt_" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
timeout -k 10 200 python -u tools/gemm_exp.py > gpurun_out/gemm_exp3.log 2>&1 || { tail -20 gpurun_out/gemm_exp3.log; exit 1; }
grep TF gpurun_out/gemm_exp3.log
timeout -k 10 300 python -u tools/gemm_nt_bench.py --cases plain > gpurun_out/gemm_nt_bench3.log 2>&1 || { tail -20 gpurun_out/gemm_nt_bench3.log; exit 1; }
tail -12 gpurun_out/gemm_nt_bench3.log
