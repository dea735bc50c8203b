export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_ab.py --arm "base:" --arm "swiglu_grid:ops.fused.SWIGLU_BWD_VARIANT=0" --arm "rope_sep:ops.fused.FUSED_ROPE_BWD=False" --rounds 4 --steps 5 > gpurun_out/step_ab1.log 2>&1 || { tail -20 gpurun_out/step_ab1.log; exit 1; }
tail -3 gpurun_out/step_ab1.log
timeout -k 10 300 python -u tools/gemm_kscan.py > gpurun_out/gemm_kscan.log 2>&1 || { tail -20 gpurun_out/gemm_kscan.log; exit 1; }
tail -3 gpurun_out/gemm_kscan.log
