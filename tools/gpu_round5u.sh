# Round-5 GPU checks, part u: forward-kernel tests incl. fwd16 (fwd_pipe = 2).
set -u -o pipefail
O=gpurun_out/r5u; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention_fwd" > $O/pytest_fwd.log 2>&1 || { tail -30 $O/pytest_fwd.log; exit 1; }
tail -1 $O/pytest_fwd.log
