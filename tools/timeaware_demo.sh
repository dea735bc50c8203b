#!/bin/bash
# BASELINE config 4 on one MI355X (no SLURM on the box): a simulated wall-clock limit via
# SLURM_JOB_END_TIME, time-aware checkpointing + async checkpoints + md5 verification, a dry-run
# resubmission, then `--resume-from-checkpoint latest` to the target step. Llama-2-7B shape with
# 8 layers so checkpoints fit the box's disk. Logs -> gpurun_out/timeaware/.
set -u
mkdir -p gpurun_out/timeaware
CK=/tmp/pyrecover_timeaware
rm -rf $CK
export PYRECOVER_RESUBMIT_DRYRUN=1 HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="--model-preset llama2-7b --n-layers 8 --synthetic-data --sequence-length 2048 --batch-size 4 \
  --training-steps 1500 --checkpoint-frequency 200 --logging-frequency 10 --checkpoint-dir $CK \
  --experiment_name ta --verify-checkpoints --async-checkpoint --timeaware-checkpointing \
  --max-kept-checkpoints 2 --resubmit requeue --num-workers 2"
export SLURM_JOB_END_TIME=$(( $(date +%s) + ${LIMIT_S:-90} ))
timeout -k 10 400 python train.py $ARGS > gpurun_out/timeaware/run1.log 2>&1 || { tail -40 gpurun_out/timeaware/run1.log; exit 1; }
grep -E "TIME CHECK|final|Checkpoint|resubmi|Training completed|stopp" gpurun_out/timeaware/run1.log | tail -15
ls -la $CK/ta > gpurun_out/timeaware/ckpts_after_run1.txt
unset SLURM_JOB_END_TIME
timeout -k 10 600 python train.py $ARGS --resume-from-checkpoint latest > gpurun_out/timeaware/run2.log 2>&1 \
  || { tail -40 gpurun_out/timeaware/run2.log; exit 1; }
grep -E "Resum|loaded|Checkpoint load|Step: 1500|Training completed" gpurun_out/timeaware/run2.log | tail -10
ls -la $CK/ta > gpurun_out/timeaware/ckpts_after_run2.txt
rm -rf $CK
