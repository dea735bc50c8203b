#!/bin/bash
# Tune hipBLASLt GEMM solutions for the bench shapes on one MI355X; result lands in gpurun_out/.
set -u
mkdir -p gpurun_out
export PRA_TUNING_TABLE=$PWD/gpurun_out/tunableop_gfx950.csv PYTORCH_TUNABLEOP_VERBOSE=1
[ -f gpurun_out/tunableop_gfx950.csv ] || cp tuning/tunableop_gfx950.csv gpurun_out/  # extend the committed table
export PRA_TUNE_MS=${PRA_TUNE_MS:-20} PRA_TUNE_ITERS=${PRA_TUNE_ITERS:-10}
timeout -k 10 1100 python bench.py --gemm-tuning tune --steps 1 --warmup 1 ${TUNE_ARGS:-} > gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -3 gpurun_out/tune.log; ls -la gpurun_out/tunableop_gfx950.csv; exit $rc
