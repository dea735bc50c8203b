# Round-5 GPU checks, part k: per-shape (grid) kernel times inside the 7B B16 step.
set -u -o pipefail
O=gpurun_out/r5k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t7b -o t -- python3 bench.py --steps 3 --warmup 3 > $O/t7b.log 2>&1 || { tail -20 $O/t7b.log; exit 1; }
python tools/trace_summary.py $(find $O/t7b -name 't_kernel_trace.csv' | head -1) --steps 2 --by-grid --top 60 > $O/trace_7b_b16_by_grid.txt 2>&1; head -50 $O/trace_7b_b16_by_grid.txt
rm -rf $O/t7b
