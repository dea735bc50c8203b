# Round-5 GPU checks, part q: per-shape step trace with the QKV projection on the NT kernel (RoPE epilogue).
set -u -o pipefail
O=gpurun_out/r5q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PYRECOVER_GEMM=w13,qkv timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t7b -o t -- python3 bench.py --steps 3 --warmup 3 > $O/t7b.log 2>&1 || { tail -20 $O/t7b.log; exit 1; }
python tools/trace_summary.py $(find $O/t7b -name 't_kernel_trace.csv' | head -1) --steps 2 --by-grid --top 30 > $O/trace_7b_b16_qkv_nt.txt 2>&1; head -30 $O/trace_7b_b16_qkv_nt.txt
rm -rf $O/t7b
