#!/bin/bash
set -u
mkdir -p gpurun_out
df -h /tmp . 2>&1 | tee gpurun_out/df.log
free -g | tee -a gpurun_out/df.log
D=${CKPT_DIR:-/tmp/pyrecover_ckpt_bench}
timeout -k 10 300 python bench_ckpt.py --n-layers 2 --dir $D --verify > gpurun_out/ckpt_small.log 2>&1; rc=$?
echo "small rc=$rc"; tail -2 gpurun_out/ckpt_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench_ckpt.py --dir $D ${CKPT_ARGS:---verify} > gpurun_out/ckpt_7b.log 2>&1; rc=$?
echo "7b rc=$rc"; tail -2 gpurun_out/ckpt_7b.log; rm -rf $D; exit $rc
