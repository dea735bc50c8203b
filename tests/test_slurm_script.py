"""submit-training-simple.sh under a fake SLURM (fake srun/scontrol/squeue on PATH, CPU training):
SIGUSR1 sent to the BATCH SHELL (what `#SBATCH --signal=B:USR1@120` does) must reach train.py,
which writes ckpt_<N>_final and requeues the job exactly once; the requeued job (SLURM_RESTART_COUNT
1) resumes from that checkpoint. Reference: submit-training-simple.sh:29-47, 135-162;
train.py:342-375."""
import os
import signal
import subprocess
import time
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

FAKE_SRUN = """#!/bin/bash
# fake srun: drop srun's own options, run the task as a child and relay signals to it
while [[ "$1" == --* ]]; do shift; done
"$@" &
CHILD=$!
trap 'kill -USR1 $CHILD' USR1
trap 'kill -TERM $CHILD' TERM
while true; do wait $CHILD; RC=$?; kill -0 $CHILD 2>/dev/null || break; done
exit $RC
"""
FAKE_SCONTROL = """#!/bin/bash
if [ "$1" = "show" ]; then echo 127.0.0.1; exit 0; fi
echo "$@" >> "$FAKE_SLURM_LOG"
echo "scontrol $*"
"""
FAKE_SQUEUE = """#!/bin/bash
echo 39:00
"""


def _fake_bin(tmp: Path) -> Path:
    b = tmp / "bin"
    b.mkdir()
    for name, body in (("srun", FAKE_SRUN), ("scontrol", FAKE_SCONTROL), ("squeue", FAKE_SQUEUE)):
        (b / name).write_text(body)
        (b / name).chmod(0o755)
    return b


def _env(tmp: Path, restart: int):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                             "SLURM_JOB_END_TIME", "SLURM_PROCID")}
    env.update(PATH=f"{_fake_bin(tmp) if not (tmp / 'bin').exists() else tmp / 'bin'}:{env['PATH']}",
               SLURM_JOB_ID="4242", SLURM_NODELIST="node0", SLURM_NNODES="1", SLURM_NTASKS_PER_NODE="1",
               SLURM_NTASKS="1", SLURM_CPUS_PER_TASK="2", SLURM_SUBMIT_DIR=str(ROOT),
               SLURM_RESTART_COUNT=str(restart), FAKE_SLURM_LOG=str(tmp / "slurm_calls.log"),
               MASTER_PORT="29999", PYTHONUNBUFFERED="1")
    return env


def _args(ckdir):
    return ["--timeaware-checkpointing", "--resubmit=requeue", "--model-preset=llama-micro", "--synthetic-data",
            "--batch-size=2", "--sequence-length=64", "--training-steps=1000000", "--exp_name=slurmtest",
            f"--checkpoint-dir={ckdir}", "--max-resubmits=3"]


def test_usr1_to_batch_shell_writes_final_checkpoint_and_requeues_once(tmp_path):
    ck = tmp_path / "ck"
    env = _env(tmp_path, 0)
    log = open(tmp_path / "job.log", "w")
    p = subprocess.Popen(["bash", str(ROOT / "submit-training-simple.sh")] + _args(ck), cwd=ROOT, env=env,
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        deadline = time.time() + 240
        # wait until the trainer is stepping (log lines every 10 steps)
        while time.time() < deadline:
            txt = (tmp_path / "job.log").read_text()
            if "Step: 20" in txt or "step 20" in txt.lower() or "| Step" in txt:
                break
            assert p.poll() is None, txt[-4000:]
            time.sleep(0.5)
        else:
            pytest.fail("trainer never started stepping:\n" + (tmp_path / "job.log").read_text()[-4000:])
        os.kill(p.pid, signal.SIGUSR1)  # to the batch shell only, like --signal=B:USR1
        rc = p.wait(timeout=180)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
        log.close()
    txt = (tmp_path / "job.log").read_text()
    assert rc == 0, txt[-4000:]
    finals = sorted((ck / "slurmtest").glob("ckpt_*_final.pt"))
    assert len(finals) == 1, (list((ck / "slurmtest").iterdir()), txt[-3000:])
    calls = (tmp_path / "slurm_calls.log").read_text().splitlines()
    assert calls == ["requeue 4242"], calls

    # the requeued job resumes from the final checkpoint; signal it again and it goes on from there
    step = int(finals[0].name.split("_")[1])
    env = _env(tmp_path, 1)
    log = open(tmp_path / "job2.log", "w")
    p = subprocess.Popen(["bash", str(ROOT / "submit-training-simple.sh")] + _args(ck), cwd=ROOT, env=env,
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        deadline = time.time() + 240
        while time.time() < deadline:
            txt = (tmp_path / "job2.log").read_text()
            if "| Step" in txt:
                break
            assert p.poll() is None, txt[-4000:]
            time.sleep(0.5)
        os.kill(p.pid, signal.SIGUSR1)
        rc = p.wait(timeout=180)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
        log.close()
    txt = (tmp_path / "job2.log").read_text()
    assert rc == 0, txt[-4000:]
    assert f"ckpt_{step}_final" in txt and "resume" in txt.lower(), txt[-3000:]
    finals2 = sorted((ck / "slurmtest").glob("ckpt_*_final.pt"), key=lambda f: int(f.name.split("_")[1]))
    assert int(finals2[-1].name.split("_")[1]) > step
    assert (tmp_path / "slurm_calls.log").read_text().splitlines() == ["requeue 4242", "requeue 4242"]


FAKE_SRUN_MULTI = """#!/bin/bash
# fake srun for SLURM_NTASKS tasks on one node: task i gets SLURM_PROCID = SLURM_LOCALID = i
while [[ "$1" == --* ]]; do shift; done
PIDS=()
for ((i = 0; i < ${SLURM_NTASKS:-1}; i++)); do
  SLURM_PROCID=$i SLURM_LOCALID=$i "$@" &
  PIDS+=($!)
done
trap 'kill -USR1 ${PIDS[@]}' USR1
trap 'kill -TERM ${PIDS[@]}' TERM
RC=0
for p in "${PIDS[@]}"; do
  while true; do wait $p; R=$?; kill -0 $p 2>/dev/null || break; done
  [ $R -ne 0 ] && RC=$R
done
exit $RC
"""


def test_two_task_slurm_launch_binds_and_trains(tmp_path):
    """The script's own multi-task path: 2 tasks (gloo on CPU), each reaches the training loop."""
    b = _fake_bin(tmp_path)
    (b / "srun").write_text(FAKE_SRUN_MULTI)
    env = _env(tmp_path, 0)
    env.update(SLURM_NTASKS="2", SLURM_NTASKS_PER_NODE="2", MASTER_PORT="29981")
    args = ["--distributed", "--model-preset=llama-micro", "--synthetic-data", "--batch-size=4",
            "--sequence-length=32", "--training-steps=3", "--exp_name=slurm2", f"--checkpoint-dir={tmp_path / 'ck'}"]
    r = subprocess.run(["bash", str(ROOT / "submit-training-simple.sh")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    txt = r.stdout + r.stderr
    assert r.returncode == 0, txt[-4000:]
    for rank in (0, 1):
        assert f"[Rank {rank}] world_size=2, local_rank={rank}, device=cpu" in txt, txt[-4000:]
        assert f"[Rank {rank}] Starting training" in txt, txt[-4000:]
    assert "Starting training!" in txt


@pytest.mark.parametrize("count,lrank,want", [(1, 3, 0), (8, 3, 3), (8, 7, 7), (4, 5, None), (2, 2, None),
                                              (0, 2, 2)])
def test_gpu_index_maps_to_a_visible_device(monkeypatch, count, lrank, want):
    """SLURM per-task isolation shows ONE device (index 0) whatever SLURM_LOCALID is; with every
    GPU visible a local rank gets its own GPU, and more local ranks than GPUs is refused (two
    ranks silently sharing a GPU would fail later inside RCCL)."""
    import torch

    from pyrecover_amd.parallel import dist as D

    monkeypatch.delenv("PYRECOVER_LOCAL_DEVICE", raising=False)
    monkeypatch.setenv("SLURM_LOCALID", str(lrank))
    monkeypatch.setattr(torch.cuda, "is_available", lambda: count > 0)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: count)
    if want is None:
        with pytest.raises(RuntimeError, match="has no GPU of its own"):
            D.gpu_index(lrank)
    else:
        assert D.gpu_index(lrank) == want
    monkeypatch.setenv("PYRECOVER_LOCAL_DEVICE", "0")
    assert D.gpu_index(lrank) == 0
