#!/bin/bash
# Development GPU session: GPU tests (optionally a subset), kernel A/Bs, default bench, kernel trace.
# usage: tools/gpu_dev_session.sh "<pytest selection>" [ab] [bench] [prof]
# Every GPU step has its own time limit; the first failure ends the session (no further GPU work).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
sel="$1"; shift
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_dev.log 2>&1 || { tail -30 gpurun_out/pytest_dev.log; exit 1; }
  tail -2 gpurun_out/pytest_dev.log
fi
for step in "$@"; do
  case "$step" in
    ab)
      timeout -k 10 180 python -u tools/swiglu_bwd_bench.py > gpurun_out/swiglu_bwd_ab.log 2>&1 || exit 1
      cat gpurun_out/swiglu_bwd_ab.log
      timeout -k 10 180 python -u tools/attn_bench.py --B 16 > gpurun_out/attn_b16.log 2>&1 || exit 1
      tail -3 gpurun_out/attn_b16.log ;;
    bench)
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_dev.log 2>&1 || exit 1
      tail -1 gpurun_out/bench_dev.log ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dev -o run -- python3 bench.py --steps 4 --warmup 2 \
        > gpurun_out/prof_dev.log 2>&1 || exit 1
      echo prof ok ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
