# Round-5 GPU checks, part ar: Llama-3-8B S2048 B1 kernel trace at HEAD.
set -u -o pipefail
O=gpurun_out/r5ar; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o t -- python3 bench.py --model llama3-8b --batch-per-gpu 1 --steps 6 --warmup 4 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
T=$(find $O/t -name 't_kernel_trace.csv' | head -1)
python tools/trace_summary.py $T --steps 5 --top 20 > $O/kernel_trace_8b_b1_head.txt 2>&1; head -16 $O/kernel_trace_8b_b1_head.txt
rm -rf $O/t
