# Round-5 GPU checks, part am: staggered split grid of the NT GEMM (C.gemm_nt_set_stagger).
set -u -o pipefail
O=gpurun_out/r5am; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gemm_nt_gpu.py > $O/pytest_nt.log 2>&1 || { tail -30 $O/pytest_nt.log; exit 1; }
tail -2 $O/pytest_nt.log
for m in 0 1 2; do
  timeout -k 10 300 python tools/gemm_nt_bench.py --cases swiglu_b,swiglu,plain --shapes w2_dgrad,w13_fwd --stagger $m > $O/nt_bench_stagger$m.log 2>&1 || { tail -20 $O/nt_bench_stagger$m.log; exit 1; }
  echo "== stagger $m"; grep -v "^/opt" $O/nt_bench_stagger$m.log | cut -c1-220
done
timeout -k 10 700 python tools/step_ab.py --arm "base:" --arm "stg1:nt.stagger=1" --arm "stg2:nt.stagger=2" \
  --arm "w2d_stg2:nt.stagger=2;ops.fused.GEMM_SITES={'w13','w2_d'}" --rounds 4 --steps 5 > $O/step_ab_7b_b16_stagger.log 2>&1 \
  || { tail -20 $O/step_ab_7b_b16_stagger.log; exit 1; }
tail -4 $O/step_ab_7b_b16_stagger.log
