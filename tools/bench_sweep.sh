#!/bin/bash
# Batch-size sweep of bench.py on one GPU (each run time-limited; stop at the first crash).
set -u
mkdir -p gpurun_out
for b in ${SWEEP_BATCHES:-2 4 8}; do
  timeout -k 10 400 python bench.py --steps ${SWEEP_STEPS:-6} --warmup 2 --batch-per-gpu $b ${SWEEP_ARGS:-} > gpurun_out/sweep_b$b.log 2>&1
  rc=$?; echo "b=$b rc=$rc"; grep metric gpurun_out/sweep_b$b.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('peak_mem_gib'))" || tail -3 gpurun_out/sweep_b$b.log
  [ $rc -eq 0 ] || exit $rc
done
