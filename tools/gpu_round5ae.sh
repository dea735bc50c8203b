# Round-5 GPU checks, part ae: the reference's default regime (Llama-3-8B, S2048, B1) through train.py
# (DataLoader, pinned H2D, logging, JSONL) next to bench.py on the same box.
set -u -o pipefail
O=gpurun_out/r5ae; mkdir -p $O
timeout -k 10 300 python bench.py --model llama3-8b --batch-per-gpu 1 --steps 30 --warmup 5 > $O/bench_8b_b1.log 2>&1 \
  || { tail -20 $O/bench_8b_b1.log; exit 1; }
tail -1 $O/bench_8b_b1.log | cut -c1-300
timeout -k 10 400 python train.py --model-preset llama3-8b --synthetic-data --batch-size 1 --sequence-length 2048 \
  --training-steps 60 --logging-frequency 10 --checkpoint-dir /tmp/pr_t8b --checkpoint-frequency 0 --experiment_name t8b \
  --metrics-jsonl $O/train_8b_b1.jsonl > $O/train_py_8b_b1.log 2>&1 || { tail -30 $O/train_py_8b_b1.log; exit 1; }
grep -E "Step|tok" $O/train_py_8b_b1.log | tail -8
