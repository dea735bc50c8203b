# Round-5 GPU checks, part x: fp32 master weights (kernel numerics, train+resume, 7B B16 bench cost).
set -u -o pipefail
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py \
  -k "adamw_master or adamw_matches" tests/test_model_gpu.py::test_train_py_model_dtypes > $O/pytest_master.log 2>&1 \
  || { tail -30 $O/pytest_master.log; exit 1; }
tail -3 $O/pytest_master.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --master-weights fp32 > $O/bench_7b_b16_master.log 2>&1 \
  || { tail -20 $O/bench_7b_b16_master.log; exit 1; }
tail -1 $O/bench_7b_b16_master.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/bench_7b_b16.log 2>&1 || { tail -20 $O/bench_7b_b16.log; exit 1; }
tail -1 $O/bench_7b_b16.log
