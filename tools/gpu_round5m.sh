# Round-5 GPU checks, part m: fused vs split backward in the 7B B16 step, with and without the AdamW update.
set -u -o pipefail
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 900 python tools/step_ab.py --rounds 3 --steps 4 --arm "split:attn.bwd_fused=0" --arm "fused:attn.bwd_fused=1" \
  --arm "split_noupd:attn.bwd_fused=0;noupdate" --arm "fused_noupd:attn.bwd_fused=1;noupdate" > $O/step_ab_fused_bwd_noupd.log 2>&1 || { tail -30 $O/step_ab_fused_bwd_noupd.log; exit 1; }
grep median $O/step_ab_fused_bwd_noupd.log
