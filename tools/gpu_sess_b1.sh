export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_ab.py --fwd --opt fwd_pipe --values 1,0 > gpurun_out/attn_ab_fwd_pipe.log 2>&1 || { tail -20 gpurun_out/attn_ab_fwd_pipe.log; exit 1; }
cat gpurun_out/attn_ab_fwd_pipe.log | grep fwd_pipe
timeout -k 10 300 python -u bench.py --batch-per-gpu 1 --steps 30 --warmup 5 > gpurun_out/bench_b1.log 2>&1 || { tail -20 gpurun_out/bench_b1.log; exit 1; }
tail -1 gpurun_out/bench_b1.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o run -- python3 bench.py --batch-per-gpu 1 --steps 6 --warmup 3 > gpurun_out/prof_b1.log 2>&1 || { tail -20 gpurun_out/prof_b1.log; exit 1; }
echo prof ok
