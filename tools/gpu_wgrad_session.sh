export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -u tools/wgrad_bench.py > gpurun_out/wgrad_bench6.log 2>&1 || exit 1
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -k wgrad -x -q --timeout 60 --timeout-method thread > gpurun_out/pt_wgrad.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/bench_wgrad2.log 2>&1 || exit 1
PYRECOVER_WGRAD=lib timeout -k 10 200 python -u bench.py > gpurun_out/bench_lib2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wgrad -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_wgrad.log 2>&1 || exit 1
