#!/bin/bash
# Round-end evidence on one MI355X: full GPU suite, smoke, default bench, kernel trace of the bench.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_final.log 2>&1 || exit 1
