# Round-5 GPU checks, part at: AdamW window by shape (before dQ at <= 4096 tokens): full GPU tests, A/B at 8B B1.
set -u -o pipefail
O=gpurun_out/r5at; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python tools/step_ab.py --arm "auto:" --arm "after_dq:attn.bwd_window=0" --rounds 8 --steps 10 \
  --model llama3-8b --batch-per-gpu 1 > $O/step_ab_8b_b1_window_auto.log 2>&1 || { tail -20 $O/step_ab_8b_b1_window_auto.log; exit 1; }
tail -2 $O/step_ab_8b_b1_window_auto.log
timeout -k 10 300 python bench.py --model llama3-8b --batch-per-gpu 1 --steps 30 --warmup 5 > $O/bench_8b_b1.log 2>&1 || { tail -20 $O/bench_8b_b1.log; exit 1; }
tail -1 $O/bench_8b_b1.log | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench_7b_b16.log 2>&1 || { tail -20 $O/bench_7b_b16.log; exit 1; }
tail -1 $O/bench_7b_b16.log | cut -c1-200
