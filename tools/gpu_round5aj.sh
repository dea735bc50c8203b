# Round-5 GPU checks, part aj: in-step A/B of the fused-epilogue GEMM sites under the XCD order:
# SwiGLU backward on the W2 data gradient (w2_d), RoPE on the QKV projection (qkv).
set -u -o pipefail
O=gpurun_out/r5aj; mkdir -p $O
timeout -k 10 600 python tools/step_ab.py --arm "base:" --arm "w2d:ops.fused.GEMM_SITES={'w13','w2_d'}" \
  --arm "qkv_w2d:ops.fused.GEMM_SITES={'w13','w2_d','qkv'}" --rounds 4 --steps 5 > $O/step_ab_7b_b16_epilogues.log 2>&1 \
  || { tail -20 $O/step_ab_7b_b16_epilogues.log; exit 1; }
tail -4 $O/step_ab_7b_b16_epilogues.log
