# Round-5 GPU checks, part o: where the AdamW window opens in the split attention backward.
set -u -o pipefail
O=gpurun_out/r5o; mkdir -p $O
timeout -k 10 900 python tools/step_ab.py --rounds 3 --steps 4 --arm "base:" --arm "early:attn.bwd_window=1" \
  --arm "early_dqplain:attn.bwd_window=1;attn.dq_pipe=0" --arm "dqplain:attn.dq_pipe=0" > $O/step_ab_7b_window.log 2>&1 || { tail -30 $O/step_ab_7b_window.log; exit 1; }
grep median $O/step_ab_7b_window.log
timeout -k 10 600 python tools/step_ab.py --model llama3-8b --batch-per-gpu 1 --rounds 4 --steps 10 --arm "base:" --arm "early:attn.bwd_window=1" \
  --arm "early_dqplain:attn.bwd_window=1;attn.dq_pipe=0" > $O/step_ab_8b_b1_window.log 2>&1 || { tail -30 $O/step_ab_8b_b1_window.log; exit 1; }
grep median $O/step_ab_8b_b1_window.log
