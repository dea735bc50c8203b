export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gemm_exp.py > gpurun_out/gemm_exp2.log 2>&1 || { tail -20 gpurun_out/gemm_exp2.log; exit 1; }
cat gpurun_out/gemm_exp2.log | grep TF
timeout -k 10 200 python -u tools/gemm_exp.py --M 12288 --N 4096 --K 32768 > gpurun_out/gemm_exp2_qkv.log 2>&1 || { tail -20 gpurun_out/gemm_exp2_qkv.log; exit 1; }
cat gpurun_out/gemm_exp2_qkv.log | grep TF
