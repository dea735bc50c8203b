# Round-5 GPU checks, part ac: in-step A/B of the opt-in attention backward variants under the XCD order.
set -u -o pipefail
O=gpurun_out/r5ac; mkdir -p $O
timeout -k 10 600 python tools/step_ab.py --arm "base:" --arm "ring:attn.dkdv_kreg=2" --arm "win1:attn.bwd_window=1" \
  --arm "fused:attn.bwd_fused=1" --rounds 4 --steps 5 > $O/step_ab_7b_b16_bwd_variants.log 2>&1 \
  || { tail -20 $O/step_ab_7b_b16_bwd_variants.log; exit 1; }
tail -5 $O/step_ab_7b_b16_bwd_variants.log
