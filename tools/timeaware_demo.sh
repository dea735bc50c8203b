#!/bin/bash
# BASELINE config 4 on one MI355X (no SLURM on the box): a simulated wall-clock limit via
# SLURM_JOB_END_TIME, time-aware checkpointing + async checkpoints + md5 verification, a dry-run
# resubmission, then `--resume-from-checkpoint latest` to the target step. Llama-2-7B shape with
# 8 layers by default so checkpoints fit the box's disk; the full-size run (TA_LAYERS=32 TA_BATCH=16,
# checkpoints of 37.7 GiB) keeps them in /dev/shm (TA_CKDIR). Logs -> gpurun_out/${TA_OUT:-timeaware}/.
set -u
OUT=gpurun_out/${TA_OUT:-timeaware}
mkdir -p $OUT
CK=${TA_CKDIR:-/tmp/pyrecover_timeaware}
rm -rf $CK
export PYRECOVER_RESUBMIT_DRYRUN=1 HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS="--model-preset llama2-7b --n-layers ${TA_LAYERS:-8} --synthetic-data --sequence-length 2048 \
  --batch-size ${TA_BATCH:-4} --training-steps ${TA_STEPS:-1500} --checkpoint-frequency ${TA_FREQ:-200} \
  --logging-frequency ${TA_LOGF:-10} --checkpoint-dir $CK \
  --experiment_name ta --verify-checkpoints --async-checkpoint --timeaware-checkpointing \
  --max-kept-checkpoints ${TA_KEEP:-2} --resubmit requeue --num-workers 2"
export SLURM_JOB_END_TIME=$(( $(date +%s) + ${LIMIT_S:-90} ))
timeout -k 10 400 python train.py $ARGS > $OUT/run1.log 2>&1 || { tail -40 $OUT/run1.log; exit 1; }
grep -E "TIME CHECK|final|Checkpoint|resubmi|Training completed|stopp|probe|max_iter" $OUT/run1.log | tail -20
ls -la --time-style=+%s $CK/ta > $OUT/ckpts_after_run1.txt
# soundness: the final checkpoint and its .md5 exist before the (simulated) wall-clock limit
fin=$(ls $CK/ta/ckpt_*_final.pt 2>/dev/null | head -1)
if [ -n "$fin" ] && [ -f "$fin.md5" ]; then
  echo "final .md5 written at $(stat -c %Y $fin.md5), limit $SLURM_JOB_END_TIME, margin $(( SLURM_JOB_END_TIME - $(stat -c %Y $fin.md5) )) s" | tee $OUT/final_md5_margin.txt
else
  echo "NO final checkpoint with .md5" | tee $OUT/final_md5_margin.txt
fi
unset SLURM_JOB_END_TIME
timeout -k 10 600 python train.py $ARGS --resume-from-checkpoint latest > $OUT/run2.log 2>&1 \
  || { tail -40 $OUT/run2.log; exit 1; }
grep -E "Resum|loaded|Checkpoint load|Step: ${TA_STEPS:-1500}|Training completed" $OUT/run2.log | tail -10
ls -la --time-style=+%s $CK/ta > $OUT/ckpts_after_run2.txt
if [ "${TA_REF:-0}" = "1" ]; then
  # bit-exact resume check: an uninterrupted run to the same step, final checkpoints compared
  last=$CK/ta/ckpt_${TA_STEPS:-1500}.pt
  [ -f $last ] || { echo "no $last"; exit 1; }
  find $CK/ta -name 'ckpt_*' ! -name "ckpt_${TA_STEPS:-1500}.pt*" -delete
  timeout -k 10 600 python train.py ${ARGS/--experiment_name ta/--experiment_name ref} > $OUT/ref.log 2>&1 \
    || { tail -40 $OUT/ref.log; exit 1; }
  timeout -k 10 300 python tools/check_weights_equality.py --optimizer $last $CK/ref/ckpt_${TA_STEPS:-1500}.pt \
    > $OUT/weights_equality.log 2>&1; echo "check_weights_equality rc=$?" >> $OUT/weights_equality.log
  tail -5 $OUT/weights_equality.log
fi
rm -rf $CK
