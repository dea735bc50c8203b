#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks pinned to GPU 0 over gloo (RCCL needs one GPU per
# rank). Exercises bench.py's distributed path (init, broadcast, bucketed async all-reduce on GPU
# tensors, max-over-ranks timing) and train.py's sharded save / preempt / resume with 2 ranks.
set -u
mkdir -p gpurun_out/dist
export PYRECOVER_LOCAL_DEVICE=0 PYRECOVER_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29511 bench.py --gpus 2 --model gpt2-small --batch-per-gpu 2 --steps 4 --warmup 2 \
  > gpurun_out/dist/bench2.log 2>&1 || { tail -30 gpurun_out/dist/bench2.log; exit 1; }
grep '"metric"' gpurun_out/dist/bench2.log
T="train.py --model-preset llama-tiny --synthetic-data --distributed --batch-size 4 --sequence-length 256 \
   --training-steps 6 --checkpoint-frequency 3 --logging-frequency 1 --use-torch-distributed-ckpt --num-workers 0"
timeout -k 10 300 $R --master-port 29512 $T --checkpoint-dir gpurun_out/dist/a > gpurun_out/dist/a.log 2>&1 \
  || { tail -30 gpurun_out/dist/a.log; exit 1; }
timeout -k 10 300 $R --master-port 29513 $T --checkpoint-dir gpurun_out/dist/b --stop-at-step 4 > gpurun_out/dist/b1.log 2>&1 \
  || { tail -30 gpurun_out/dist/b1.log; exit 1; }
timeout -k 10 300 $R --master-port 29514 $T --checkpoint-dir gpurun_out/dist/b --resume-from-checkpoint latest \
  > gpurun_out/dist/b2.log 2>&1 || { tail -30 gpurun_out/dist/b2.log; exit 1; }
timeout -k 10 120 python tools/check_weights_equality.py gpurun_out/dist/a/default-exp/ckpt_6 \
  gpurun_out/dist/b/default-exp/ckpt_6 --distributed --optimizer --tolerance 0
timeout -k 10 300 $R --master-port 29515 bench.py --gpus 2 --model gpt2-small --batch-per-gpu 2 --steps 4 --warmup 2 \
  --allreduce xgmi > gpurun_out/dist/bench2_xgmi.log 2>&1 || { tail -30 gpurun_out/dist/bench2_xgmi.log; exit 1; }
grep '"metric"' gpurun_out/dist/bench2_xgmi.log
