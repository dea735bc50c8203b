export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/gemm_exp.py > gpurun_out/gemm_exp.log 2>&1 || { tail -20 gpurun_out/gemm_exp.log; exit 1; }
cat gpurun_out/gemm_exp.log | grep TF
ATTN_ARGS="--B 16" timeout -k 10 900 bash tools/attn_prof.sh || exit 1
python3 tools/pmc_summary.py gpurun_out/attn/pmc1 gpurun_out/attn/pmc2 > gpurun_out/attn/pmc_summary.txt 2>&1 || true
tail -40 gpurun_out/attn/pmc_summary.txt
