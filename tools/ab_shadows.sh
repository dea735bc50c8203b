#!/bin/bash
# A/B of the transposed weight shadows (PRA_WEIGHT_SHADOWS=1 default vs 0), interleaved runs.
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for s in 1 0; do
    PRA_WEIGHT_SHADOWS=$s timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${AB_ARGS:-} > gpurun_out/ab_s${s}_$i.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "shadows=$s rc=$rc"; tail -5 gpurun_out/ab_s${s}_$i.log; exit $rc; }
    echo "shadows=$s run=$i $(grep metric gpurun_out/ab_s${s}_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gib"])')"
  done
done
