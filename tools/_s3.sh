set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --phase-timing > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
PYRECOVER_TN_WGRAD=0 timeout -k 10 400 python bench.py --steps 6 > gpurun_out/bench_notn.log 2>&1
tail -1 gpurun_out/bench_notn.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof.log 2>&1
echo prof ok
