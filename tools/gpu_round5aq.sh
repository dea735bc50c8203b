# Round-5 GPU checks, part aq: train.py at Llama-3-8B S2048 B1 with 0 / 1 / 2 DataLoader workers.
set -u -o pipefail
O=gpurun_out/r5aq; mkdir -p $O
for w in 0 1 2; do
  timeout -k 10 400 python train.py --model-preset llama3-8b --synthetic-data --batch-size 1 --sequence-length 2048 \
    --training-steps 60 --logging-frequency 10 --checkpoint-dir /tmp/pr_t8b_$w --checkpoint-frequency 0 --experiment_name t \
    --num-workers $w > $O/train_8b_b1_w$w.log 2>&1 || { tail -30 $O/train_8b_b1_w$w.log; exit 1; }
  echo "workers $w: $(grep -E 'Step: (30|40|50|60) ' $O/train_8b_b1_w$w.log | sed -E 's/.*Tokens per second: ([0-9.]+).*/\1/' | tr '\n' ' ')"
done
