#!/bin/bash
#SBATCH --job-name=pyrecover-amd
#SBATCH --nodes=1
#SBATCH --ntasks-per-node=8
#SBATCH --gpus-per-node=8
#SBATCH --cpus-per-task=16
#SBATCH --time=00:40:00
#SBATCH --signal=B:USR1@120
#SBATCH --requeue
#SBATCH --output=logs/%x-%j.out
#
# MI355X SLURM launcher with the reference's script flags (reference submit-training-simple.sh):
#   --distributed --exp_name=NAME --continue --use_torch_distributed_ckpt --timeaware-checkpointing
#   --use_flash_attention --log-loss-to-csv --fused-optimizer --compile --sequence-length=N
#   --profile-nsys (rocprofv3 on MI355X)
# plus: --async-checkpoint, --resubmit=requeue|chain, --model-preset=NAME, --synthetic-data,
#       --batch-size=N, --training-steps=N
#       --checkpoint-dir=DIR, --max-resubmits=N
# Fixes vs the reference: --sequence-length is passed with its flag name, the
# distributed run uses one task per GPU, SIGUSR1 ahead of the limit triggers the final checkpoint.
#
# Preemption path: `--signal=B:USR1@120` delivers SIGUSR1 to THIS batch shell 120 s before the
# limit. The shell runs srun in the background and waits on it; its trap forwards the signal to
# srun, which relays it to every task, where train.py --handle-signals writes ckpt_<N>_final and
# (with --resubmit) requeues the job. A requeued job sees SLURM_RESTART_COUNT > 0 and resumes.
set -euo pipefail
cd "${SLURM_SUBMIT_DIR:-.}"
mkdir -p logs

# ---- job end time for time-aware checkpointing (reference :29-47) ----
if [ -n "${SLURM_JOB_START_TIME:-}" ] && [ -n "${SLURM_TIMELIMIT:-}" ]; then
  START=$SLURM_JOB_START_TIME
  if ! [[ "$START" =~ ^[0-9]+$ ]]; then START=$(date -d "$START" +%s); fi
  LIMIT_MIN=$SLURM_TIMELIMIT
  if ! [[ "$LIMIT_MIN" =~ ^[0-9]+$ ]]; then
    LIMIT_MIN=$(echo "$LIMIT_MIN" | awk -F'[-:]' '{ if (NF==4) print $1*1440+$2*60+$3; else if (NF==3) print $1*60+$2; else print $1 }')
  fi
  export SLURM_JOB_END_TIME=$((START + LIMIT_MIN * 60))
elif [ -n "${SLURM_JOB_ID:-}" ]; then
  LEFT=$(squeue -h -j "$SLURM_JOB_ID" -o %L 2>/dev/null || true)
  if [ -n "$LEFT" ]; then
    export SLURM_JOB_END_TIME=$(python3 -c "import sys,time; sys.path.insert(0,'.'); from pyrecover_amd.timelimit import _parse_slurm_duration as p; print(int(time.time()+(p('$LEFT') or 0)))")
  fi
fi
echo "SLURM_JOB_END_TIME=${SLURM_JOB_END_TIME:-unset}"

# ---- fixed run configuration (reference :122-127) ----
TRAINING_STEPS=3000
LOGGING_FREQ=10
CHECKPOINT_FREQ=1000
GLOBAL_BATCH_SIZE=8
ITER_TIME=1
CKPT_TIME=10
SEQ_LEN=2048
EXP_NAME="default-exp"
EXTRA=()
PROFILE=0
for arg in "$@"; do
  case "$arg" in
    --distributed) EXTRA+=(--distributed) ;;
    --exp_name=*) EXP_NAME="${arg#*=}" ;;
    --continue) EXTRA+=(--resume-from-checkpoint=latest) ;;
    --use_torch_distributed_ckpt) EXTRA+=(--use-torch-distributed-ckpt) ;;
    --timeaware-checkpointing) EXTRA+=(--timeaware-checkpointing --handle-signals) ;;
    --use_flash_attention) EXTRA+=(--use_flash_attention) ;;
    --log-loss-to-csv) EXTRA+=(--log-loss-to-csv) ;;
    --fused-optimizer) EXTRA+=(--fused-optimizer) ;;
    --compile) EXTRA+=(--compile) ;;
    --sequence-length=*) SEQ_LEN="${arg#*=}" ;;
    --batch-size=*) GLOBAL_BATCH_SIZE="${arg#*=}" ;;
    --training-steps=*) TRAINING_STEPS="${arg#*=}" ;;
    --model-preset=*) EXTRA+=(--model-preset "${arg#*=}") ;;
    --synthetic-data) EXTRA+=(--synthetic-data) ;;
    --async-checkpoint) EXTRA+=(--async-checkpoint) ;;
    --resubmit=*) EXTRA+=(--resubmit "${arg#*=}" --resubmit-script "$0") ;;
    --max-resubmits=*) EXTRA+=(--max-resubmits "${arg#*=}") ;;
    --checkpoint-dir=*) EXTRA+=(--checkpoint-dir "${arg#*=}") ;;
    --profile-nsys|--profile-rocprof) PROFILE=1 ;;
    *) echo "unknown argument $arg"; exit 2 ;;
  esac
done
# a requeued/chained job resumes automatically
if [ "${SLURM_RESTART_COUNT:-0}" -gt 0 ] || [ "${PYRECOVER_RESUBMIT_COUNT:-0}" -gt 0 ]; then
  EXTRA+=(--resume-from-checkpoint=latest)
fi
export PYRECOVER_SCRIPT_ARGS="$*"

export MASTER_ADDR=$(scontrol show hostnames "$SLURM_NODELIST" | head -n 1)
export MASTER_PORT=${MASTER_PORT:-12345}
export WORLD_SIZE=$((SLURM_NNODES * SLURM_NTASKS_PER_NODE))
export HSA_ENABLE_IPC_MODE_LEGACY=0
export OMP_NUM_THREADS=${SLURM_CPUS_PER_TASK:-8}

CMD=(python3 train.py --sequence-length "$SEQ_LEN" --batch-size "$GLOBAL_BATCH_SIZE"
     --training-steps "$TRAINING_STEPS" --logging-frequency "$LOGGING_FREQ"
     --checkpoint-frequency "$CHECKPOINT_FREQ" --experiment_name "$EXP_NAME"
     --default-iter-time "$ITER_TIME" --default-ckpt-time "$CKPT_TIME" --verify-checkpoints "${EXTRA[@]}")

if [ "$PROFILE" -eq 1 ]; then
  # rocprofv3 collects kernels inside the --profile window (roctx regions, steps 10-12)
  CMD=(rocprofv3 --kernel-trace --stats --marker-trace --output-format csv -d "logs/rocprof-$SLURM_JOB_ID" --
       "${CMD[@]}" --profile)
fi
echo "Running: ${CMD[*]}"
# one task per GPU; SLURM_PROCID selects the rank. By default every node GPU is visible to every
# task (reference dist_utils.py:47,55) and SLURM_LOCALID selects the device; this is what peer IPC
# (--allreduce xgmi) needs. PYRECOVER_GPU_BIND=closest isolates one GPU per task instead
# (--gpus-per-task=1 --gpu-bind=closest): each task then sees device 0 and uses it
# (pyrecover_amd/parallel/dist.py gpu_index). srun runs in the background so the trap below can
# forward SIGUSR1/SIGTERM while the shell waits.
SRUN_OPTS=(--kill-on-bad-exit=1)
if [ -n "${PYRECOVER_GPU_BIND:-}" ]; then
  SRUN_OPTS+=(--gpus-per-task=1 "--gpu-bind=${PYRECOVER_GPU_BIND}")
fi
srun "${SRUN_OPTS[@]}" "${CMD[@]}" &
SRUN_PID=$!
forward() {
  echo "batch shell: received $1, forwarding to the job step (srun pid $SRUN_PID)"
  kill -s "$1" "$SRUN_PID" 2>/dev/null || true
}
trap 'forward USR1' USR1
trap 'forward TERM' TERM
RC=0
# `wait` returns early (status > 128) whenever a trapped signal arrives: keep waiting for srun
while true; do
  set +e
  wait "$SRUN_PID"
  RC=$?
  set -e
  if ! kill -0 "$SRUN_PID" 2>/dev/null; then break; fi
done
echo "job step exited with status $RC"
exit "$RC"
