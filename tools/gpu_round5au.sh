# Round-5 GPU checks, part au: AdamW window before dQ at Llama-3-8B S8192 B1 and Llama-3-8B S2048 B4.
set -u -o pipefail
O=gpurun_out/r5au; mkdir -p $O
timeout -k 10 400 python tools/step_ab.py --arm "after_dq:attn.bwd_window=0" --arm "before_dq:attn.bwd_window=1" --rounds 6 --steps 5 \
  --model llama3-8b --seq-len 8192 --batch-per-gpu 1 > $O/step_ab_8b_s8192_window.log 2>&1 || { tail -20 $O/step_ab_8b_s8192_window.log; exit 1; }
tail -2 $O/step_ab_8b_s8192_window.log
timeout -k 10 400 python tools/step_ab.py --arm "after_dq:attn.bwd_window=0" --arm "before_dq:attn.bwd_window=1" --rounds 6 --steps 5 \
  --model llama3-8b --batch-per-gpu 4 > $O/step_ab_8b_b4_window.log 2>&1 || { tail -20 $O/step_ab_8b_b4_window.log; exit 1; }
tail -2 $O/step_ab_8b_b4_window.log
