# Round-5 GPU checks, part r: per-kernel trace of Llama-3-8B S8192 B1 (BASELINE config 5).
set -u -o pipefail
O=gpurun_out/r5r; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/t8 -o t -- python3 bench.py --model llama3-8b --seq-len 8192 --batch-per-gpu 1 --steps 3 --warmup 3 > $O/t8.log 2>&1 || { tail -20 $O/t8.log; exit 1; }
python tools/trace_summary.py $(find $O/t8 -name 't_kernel_trace.csv' | head -1) --steps 2 --by-grid --top 40 > $O/trace_8b_s8192_b1.txt 2>&1; head -40 $O/trace_8b_s8192_b1.txt
rm -rf $O/t8
timeout -k 10 400 python bench.py --model llama3-8b --seq-len 8192 --batch-per-gpu 1 --steps 10 --warmup 3 > $O/bench_8b_s8192.log 2>&1 || { tail -20 $O/bench_8b_s8192.log; exit 1; }
tail -1 $O/bench_8b_s8192.log | cut -c1-300
