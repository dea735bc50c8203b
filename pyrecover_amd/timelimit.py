"""SLURM wall-clock awareness (declared but missing in the reference: pyrecover/__init__.py:6-7).

* :func:`get_job_end_time` - ``SLURM_JOB_END_TIME`` (set by our submit script), else the job's
  end time from ``squeue``/``scontrol``, else None.
* :func:`get_remaining_time` - seconds until that end time (None if unknown).
* :class:`TimeAwareStopper` - the reference's stop rule (train.py:164-232, 298-307, 334-337):
  stop when ``remaining < max_iter + max_ckpt + buffer`` with ``buffer = 10*iter + 2*ckpt``
  initially and ``5*max_iter + 1*max_ckpt`` after the first step; maxima are running maxima.
  Extended with a byte-based estimate of the final save (so the budget is sound before any save
  has completed), the in-flight async-checkpoint drain time, the one-step-late distributed stop
  flag, and a signal path (SIGUSR1/SIGTERM, e.g. ``#SBATCH --signal=B:USR1@120``) that requests a
  stop immediately.
* :func:`monitor_timelimit` - optional background thread that sets a flag near the deadline.
"""
from __future__ import annotations

import logging
import os
import re
import signal
import subprocess
import threading
import time
from typing import Callable, Optional

logger = logging.getLogger("pyrecover")


def _parse_slurm_duration(s: str) -> Optional[float]:
    """'D-HH:MM:SS' | 'HH:MM:SS' | 'MM:SS' | 'MM' -> seconds."""
    s = s.strip()
    if not s or s in ("UNLIMITED", "INVALID", "NOT_SET"):
        return None
    days = 0
    if "-" in s:
        d, s = s.split("-", 1)
        days = int(d)
    parts = [int(p) for p in s.split(":")]
    if len(parts) == 3:
        h, m, sec = parts
    elif len(parts) == 2:
        h, m, sec = 0, parts[0], parts[1]
    else:
        h, m, sec = 0, parts[0], 0
    return float(days * 86400 + h * 3600 + m * 60 + sec)


def get_job_end_time(query_scheduler: bool = True) -> Optional[float]:
    v = os.environ.get("SLURM_JOB_END_TIME")
    if v:
        try:
            return float(v)
        except ValueError:
            pass
    job = os.environ.get("SLURM_JOB_ID")
    if not (query_scheduler and job):
        return None
    try:
        out = subprocess.run(["squeue", "-h", "-j", job, "-o", "%L"], capture_output=True, text=True, timeout=10)
        left = _parse_slurm_duration(out.stdout) if out.returncode == 0 else None
        if left is not None:
            return time.time() + left
    except (OSError, subprocess.SubprocessError):
        pass
    return None


def get_remaining_time(end_time: Optional[float] = None, now: Optional[float] = None) -> Optional[float]:
    end = end_time if end_time is not None else get_job_end_time()
    if end is None:
        return None
    return end - (time.time() if now is None else now)


class TimeAwareStopper:
    """The reference's stop rule plus the terms it lacks.

    * ``max_iter`` / ``max_ckpt``: running maxima of observed iteration / save times, starting at
      the ``--default-iter-time`` / ``--default-ckpt-time`` priors (reference train.py:167-176).
    * ``ckpt_estimate``: the predicted cost of the FINAL save from the bytes it writes and measured
      write / MD5 rates (:class:`pyrecover_amd.ckpt.core.SaveCostModel`). The reference only
      learns a save's cost after one has completed, so a job whose first save is the final one is
      budgeted at the 10 s prior however large the model; the budget uses
      ``max(max_ckpt, ckpt_estimate)``.
    * ``inflight_drain``: what an in-flight async save (and its deferred digest) still needs
      before the final save can start / the job can exit.
    * ``extra_iters``: iterations between rank 0's decision and the stop (1 with the one-step-late
      distributed stop flag of the trainer).
    """
    ITER_MULT_INIT, CKPT_MULT_INIT = 10, 2
    ITER_MULT, CKPT_MULT = 5, 1

    def __init__(self, default_iter_time: float = 1.0, default_ckpt_time: float = 10.0,
                 end_time: Optional[float] = None, clock: Callable[[], float] = time.time,
                 install_signals: bool = False):
        self.max_iter = float(default_iter_time)
        self.max_ckpt = float(default_ckpt_time)
        self.ckpt_estimate = 0.0
        self.end_time = end_time
        self.clock = clock
        self.inflight_drain = 0.0  # seconds an in-flight async checkpoint still needs
        self.extra_iters = 0
        self.signaled = False
        self._stepped = False  # the reference switches to the steady-state buffer after step 1
        if install_signals:
            self.install_signal_handlers()

    @property
    def ckpt_budget(self) -> float:
        return max(self.max_ckpt, self.ckpt_estimate)

    @property
    def buffer(self) -> float:
        if not self._stepped:
            return self.ITER_MULT_INIT * self.max_iter + self.CKPT_MULT_INIT * self.ckpt_budget
        return self.ITER_MULT * self.max_iter + self.CKPT_MULT * self.ckpt_budget

    @property
    def threshold(self) -> float:
        return (1 + self.extra_iters) * self.max_iter + self.ckpt_budget + self.buffer + self.inflight_drain

    def remaining(self) -> Optional[float]:
        if self.end_time is None:
            return None
        return self.end_time - self.clock()

    def should_stop(self) -> bool:
        if self.signaled:
            return True
        rem = self.remaining()
        return rem is not None and rem < self.threshold

    def update_iter(self, iter_time: float) -> bool:
        changed = iter_time > self.max_iter
        self.max_iter = max(self.max_iter, iter_time)
        self._stepped = True
        return changed

    def update_ckpt(self, ckpt_time: float) -> bool:
        changed = ckpt_time > self.max_ckpt
        self.max_ckpt = max(self.max_ckpt, ckpt_time)
        return changed

    def set_ckpt_estimate(self, seconds: float) -> bool:
        """The current byte-based prediction of the final save (not a running maximum: measured
        rates replace the startup probe's as saves complete). True when the budget grew."""
        before = self.ckpt_budget
        self.ckpt_estimate = float(seconds)
        return self.ckpt_budget > before + 1e-9

    def install_signal_handlers(self, signals=(signal.SIGUSR1, signal.SIGTERM)):
        def handler(signum, frame):
            logger.warning(f"received signal {signum}: requesting checkpoint-and-stop")
            self.signaled = True

        for s in signals:
            try:
                signal.signal(s, handler)
            except (ValueError, OSError):  # not main thread / unsupported
                pass


def monitor_timelimit(threshold_s: float, callback: Optional[Callable[[], None]] = None,
                      end_time: Optional[float] = None, poll_s: float = 5.0) -> threading.Event:
    """Start a daemon thread that sets (and returns) an Event once fewer than ``threshold_s``
    seconds remain; ``callback`` is invoked once at that point."""
    ev = threading.Event()
    end = end_time if end_time is not None else get_job_end_time()

    def run():
        while not ev.is_set():
            rem = get_remaining_time(end)
            if rem is not None and rem < threshold_s:
                ev.set()
                if callback is not None:
                    callback()
                return
            time.sleep(poll_s)

    if end is not None:
        threading.Thread(target=run, name="pyrecover-timelimit", daemon=True).start()
    return ev
