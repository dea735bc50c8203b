# Round-5 GPU checks, part ak: SwiGLU-backward epilogue with row-block loads in flight (epi2_pipe):
# numerics, kernel bench against hipBLASLt + the separate kernel, in-step A/B of the w2_d site.
set -u -o pipefail
O=gpurun_out/r5ak; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gemm_nt_gpu.py > $O/pytest_nt.log 2>&1 || { tail -30 $O/pytest_nt.log; exit 1; }
tail -2 $O/pytest_nt.log
timeout -k 10 300 python tools/gemm_nt_bench.py --cases swiglu_b,plain --shapes w2_dgrad > $O/nt_bench_swiglu_b.log 2>&1 || { tail -20 $O/nt_bench_swiglu_b.log; exit 1; }
grep -v "^/opt" $O/nt_bench_swiglu_b.log
timeout -k 10 600 python tools/step_ab.py --arm "base:" --arm "w2d:ops.fused.GEMM_SITES={'w13','w2_d'}" --rounds 5 --steps 5 > $O/step_ab_7b_b16_w2d.log 2>&1 \
  || { tail -20 $O/step_ab_7b_b16_w2d.log; exit 1; }
tail -3 $O/step_ab_7b_b16_w2d.log
