#!/bin/bash
# One GPU-box session: tests -> smoke -> bench -> (optional) rocprof. Every GPU step has its own
# timeout; a crash/timeout (rc other than 0/1) stops the session (no further GPU work).
# usage: tools/gpu_session.sh [tests] [smoke] [bench] [prof] ...
set -u
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
      echo "tests rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
      echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py ${PROF_ARGS:---steps 2 --warmup 1} > gpurun_out/prof.log 2>&1; rc=$?
      echo "prof rc=$rc"; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
