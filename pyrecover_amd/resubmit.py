"""Automatic SLURM resubmission after a time-aware stop (declared but missing in the reference:
pyrecover/__init__.py:6).

Two mechanisms, selected by :func:`setup_resubmission`:

* ``requeue``: ``scontrol requeue $SLURM_JOB_ID`` (needs ``#SBATCH --requeue``); the job restarts
  with the same script, which passes ``--resume-from-checkpoint=latest``; the limit counts
  ``SLURM_RESTART_COUNT``, which SLURM increments on every requeue;
* ``chain``: ``sbatch --dependency=afterany:$SLURM_JOB_ID <script> <args>`` submits a successor
  that starts when this job ends.

Only rank 0 acts; commands are built by :func:`resubmit_command` (pure, unit-tested) and run
with a timeout. ``PYRECOVER_RESUBMIT_DRYRUN=1`` logs instead of executing.
"""
from __future__ import annotations

import logging
import os
import shlex
import subprocess
from dataclasses import dataclass, field
from typing import List, Optional

logger = logging.getLogger("pyrecover")


@dataclass
class ResubmitConfig:
    mode: str = "none"  # none | requeue | chain
    script: Optional[str] = None
    script_args: List[str] = field(default_factory=list)
    max_resubmits: int = 10


_CFG = ResubmitConfig()


def setup_resubmission(mode: str = "requeue", script: Optional[str] = None, script_args=None,
                       max_resubmits: int = 10) -> ResubmitConfig:
    global _CFG
    if mode not in ("none", "requeue", "chain"):
        raise ValueError(f"unknown resubmission mode {mode!r}")
    _CFG = ResubmitConfig(mode, script, list(script_args or []), max_resubmits)
    return _CFG


def resubmit_command(cfg: ResubmitConfig, env=None) -> Optional[List[str]]:
    env = os.environ if env is None else env
    job = env.get("SLURM_JOB_ID")
    if cfg.mode == "none" or not job:
        return None
    # requeue restarts the same job, and SLURM counts those restarts itself; chain submits a new
    # job, which carries the count in its environment
    if cfg.mode == "requeue":
        count = int(env.get("SLURM_RESTART_COUNT", "0") or 0)
    else:
        count = int(env.get("PYRECOVER_RESUBMIT_COUNT", "0") or 0)
    if count >= cfg.max_resubmits:
        return None
    if cfg.mode == "requeue":
        return ["scontrol", "requeue", job]
    if not cfg.script:
        raise ValueError("chain resubmission needs the batch script path")
    return ["sbatch", f"--dependency=afterany:{job}", f"--export=ALL,PYRECOVER_RESUBMIT_COUNT={count + 1}",
            cfg.script] + list(cfg.script_args)


def maybe_resubmit(rank: int = 0, cfg: Optional[ResubmitConfig] = None) -> bool:
    cfg = cfg or _CFG
    if rank != 0:
        return False
    cmd = resubmit_command(cfg)
    if cmd is None:
        return False
    if os.environ.get("PYRECOVER_RESUBMIT_DRYRUN") == "1":
        logger.info("[resubmit dry-run] " + " ".join(shlex.quote(c) for c in cmd))
        return True
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
        if r.returncode != 0:
            logger.error(f"resubmission failed ({r.returncode}): {r.stderr.strip()}")
            return False
        logger.info(f"resubmitted: {' '.join(cmd)} -> {r.stdout.strip()}")
        return True
    except (OSError, subprocess.SubprocessError) as e:
        logger.error(f"resubmission failed: {e}")
        return False
