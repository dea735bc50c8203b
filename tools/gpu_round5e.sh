# Round-5 GPU checks, part e: HEAD kernel traces of the 7B B16 and Llama-3-8B B1 steps.
set -u
O=gpurun_out/r5e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t7b -o t -- python3 bench.py --steps 3 --warmup 3 > $O/t7b.log 2>&1 || { tail -20 $O/t7b.log; exit 1; }
python tools/trace_summary.py $(find $O/t7b -name 't_kernel_trace.csv' | head -1) --steps 2 > $O/trace_7b_b16.txt 2>&1; head -30 $O/trace_7b_b16.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t8b -o t -- python3 bench.py --model llama3-8b --batch-per-gpu 1 --steps 6 --warmup 4 > $O/t8b.log 2>&1 || { tail -20 $O/t8b.log; exit 1; }
python tools/trace_summary.py $(find $O/t8b -name 't_kernel_trace.csv' | head -1) --steps 4 > $O/trace_8b_b1.txt 2>&1; head -30 $O/trace_8b_b1.txt
rm -rf $O/t7b $O/t8b
