# Round-5 GPU checks, part ag: secondary configs at HEAD (XCD-grouped attention order).
set -u -o pipefail
O=gpurun_out/r5ag; mkdir -p $O
timeout -k 10 300 python bench.py --model llama3-8b --seq-len 8192 --batch-per-gpu 1 --steps 10 --warmup 3 > $O/bench_8b_s8192.log 2>&1 || { tail -20 $O/bench_8b_s8192.log; exit 1; }
tail -1 $O/bench_8b_s8192.log | cut -c1-200
timeout -k 10 300 python bench.py --model gpt2-medium --steps 20 --warmup 5 > $O/bench_gpt2m_b16.log 2>&1 || { tail -20 $O/bench_gpt2m_b16.log; exit 1; }
tail -1 $O/bench_gpt2m_b16.log | cut -c1-200
timeout -k 10 300 python bench.py --model llama3-8b --steps 10 --warmup 3 > $O/bench_8b_b16.log 2>&1 || { tail -20 $O/bench_8b_b16.log; exit 1; }
tail -1 $O/bench_8b_b16.log | cut -c1-200
timeout -k 10 300 python bench.py --batch-per-gpu 1 --steps 30 --warmup 5 > $O/bench_7b_b1.log 2>&1 || { tail -20 $O/bench_7b_b1.log; exit 1; }
tail -1 $O/bench_7b_b1.log | cut -c1-200
