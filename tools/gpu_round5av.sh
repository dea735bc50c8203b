# Round-5 GPU checks, part av: fused attention backward at batch 1 (8B, 7B S2048) against the split default.
set -u -o pipefail
O=gpurun_out/r5av; mkdir -p $O
timeout -k 10 400 python tools/step_ab.py --arm "split:" --arm "fused:attn.bwd_fused=1" --rounds 8 --steps 10 \
  --model llama3-8b --batch-per-gpu 1 > $O/step_ab_8b_b1_fused.log 2>&1 || { tail -20 $O/step_ab_8b_b1_fused.log; exit 1; }
tail -2 $O/step_ab_8b_b1_fused.log
timeout -k 10 400 python tools/step_ab.py --arm "split:" --arm "fused:attn.bwd_fused=1" --rounds 6 --steps 10 \
  --model llama2-7b --batch-per-gpu 1 > $O/step_ab_7b_b1_fused.log 2>&1 || { tail -20 $O/step_ab_7b_b1_fused.log; exit 1; }
tail -2 $O/step_ab_7b_b1_fused.log
