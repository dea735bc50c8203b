# Round-5 GPU checks, part ab: 7B B16 bench and kernel trace with the XCD-grouped attention order.
set -u -o pipefail
O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_7b_b16.log 2>&1 || { tail -20 $O/bench_7b_b16.log; exit 1; }
tail -1 $O/bench_7b_b16.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t7b -o t -- python3 bench.py --steps 3 --warmup 3 > $O/t7b.log 2>&1 || { tail -20 $O/t7b.log; exit 1; }
T=$(find $O/t7b -name 't_kernel_trace.csv' | head -1)
python tools/trace_summary.py $T --steps 2 --top 25 > $O/kernel_trace_7b_b16_head.txt 2>&1; head -20 $O/kernel_trace_7b_b16_head.txt
rm -rf $O/t7b
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_7b_b16_2.log 2>&1 || { tail -20 $O/bench_7b_b16_2.log; exit 1; }
tail -1 $O/bench_7b_b16_2.log
