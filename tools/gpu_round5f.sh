# Round-5 GPU checks, part f: AdamW side stream on a CU-masked queue (opt.cu_share) and scheduling.
set -u
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 400 python tools/step_ab.py --model llama3-8b --batch-per-gpu 1 --rounds 4 --steps 10 \
  --arm "base:" --arm "cu4:opt.cu_share=4" --arm "cu8:opt.cu_share=8" --arm "cu2:opt.cu_share=2" \
  --arm "eager_cu4:optim.adamw.OPT_SCHED='eager';opt.cu_share=4" --arm "eager:optim.adamw.OPT_SCHED='eager'" \
  --arm "noupdate:noupdate" > $O/step_ab_8b_b1_cushare.log 2>&1 || { tail -30 $O/step_ab_8b_b1_cushare.log; exit 1; }
grep median $O/step_ab_8b_b1_cushare.log
timeout -k 10 600 python tools/step_ab.py --rounds 3 --steps 4 \
  --arm "base:" --arm "cu4:opt.cu_share=4" --arm "cu8:opt.cu_share=8" \
  --arm "eager_cu8:optim.adamw.OPT_SCHED='eager';opt.cu_share=8" --arm "noupdate:noupdate" > $O/step_ab_7b_cushare.log 2>&1 || { tail -30 $O/step_ab_7b_cushare.log; exit 1; }
grep median $O/step_ab_7b_cushare.log
