#!/bin/bash
# Peak-memory / throughput headroom sweep on one MI355X (288 GB HBM): bench.py at growing batch per
# GPU for the 7B S2048 and Llama-3-8B S8192 configs (BASELINE configs 3 and 5), each run in its own
# process; a run that ends in an out-of-memory error records it and the sweep goes on, any other
# failure (time limit, abort, fault) ends the sweep.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
out=gpurun_out/mem_headroom.log
: > "$out"
run() {  # model seq batch
  echo "== $1 S$2 B$3" >> "$out"
  timeout -k 10 240 python -u bench.py --model "$1" --seq-len "$2" --batch-per-gpu "$3" --steps 3 --warmup 2 \
    > gpurun_out/mem_run.log 2>&1
  rc=$?
  grep -h '"metric"' gpurun_out/mem_run.log >> "$out"
  if [ $rc -ne 0 ]; then
    if grep -q "OutOfMemoryError\|out of memory" gpurun_out/mem_run.log; then
      echo "OOM (rc $rc)" >> "$out"
      return 0
    fi
    echo "FAILED rc $rc" >> "$out"
    tail -5 gpurun_out/mem_run.log >> "$out"
    return 1
  fi
}
run llama2-7b 2048 16 && run llama2-7b 2048 20 && run llama2-7b 2048 24 &&
  run llama3-8b 8192 1 && run llama3-8b 8192 2 && run llama3-8b 8192 3 && run llama3-8b 8192 4
