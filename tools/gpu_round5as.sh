# Round-5 GPU checks, part as: AdamW window before the dQ kernel at Llama-3-8B B1 (and GPT-2-medium B16).
set -u -o pipefail
O=gpurun_out/r5as; mkdir -p $O
timeout -k 10 400 python tools/step_ab.py --arm "base:" --arm "win1:attn.bwd_window=1" --rounds 8 --steps 10 \
  --model llama3-8b --batch-per-gpu 1 > $O/step_ab_8b_b1_window.log 2>&1 || { tail -20 $O/step_ab_8b_b1_window.log; exit 1; }
tail -2 $O/step_ab_8b_b1_window.log
timeout -k 10 400 python tools/step_ab.py --arm "base:" --arm "win1:attn.bwd_window=1" --rounds 6 --steps 10 \
  --model llama2-7b --batch-per-gpu 1 > $O/step_ab_7b_b1_window.log 2>&1 || { tail -20 $O/step_ab_7b_b1_window.log; exit 1; }
tail -2 $O/step_ab_7b_b1_window.log
