"""hipBLASLt solution selection via PyTorch TunableOp.

The plain library GEMMs (QKV/O/W13/W2/output projections, their dgrad and wgrad) go through
hipBLASLt. Its default heuristic pick is not always the fastest kernel for our shapes, so we
benchmark the candidate solutions ONCE on an MI355X (``mode="tune"``) and commit the resulting
table under ``tuning/``; every later run replays it without tuning (``mode="auto"``/``"use"``).
The table records the ROCm / hipBLASLt versions and GPU arch; TunableOp ignores entries that do
not match the running stack, so a stale table can only cost speed, never correctness.
"""
from __future__ import annotations

import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TABLE = os.environ.get("PRA_TUNING_TABLE", os.path.join(ROOT, "tuning", "tunableop_gfx950.csv"))


def configure_gemm_tuning(mode: str = "auto", table: str = TABLE) -> bool:
    """Must run before the first GEMM. Returns True if TunableOp is active."""
    import torch

    if mode == "off" or not torch.cuda.is_available():
        return False
    to = torch.cuda.tunable
    if mode == "tune":
        os.makedirs(os.path.dirname(table), exist_ok=True)
        to.enable(True)
        to.tuning_enable(True)
        to.set_max_tuning_duration(int(os.environ.get("PRA_TUNE_MS", "60")))
        to.set_max_tuning_iterations(int(os.environ.get("PRA_TUNE_ITERS", "40")))
        # rank-specific output file is appended by torch when distributed; single-GPU tuning only
        to.set_filename(table, insert_device_ordinal=False)
        if os.path.exists(table):  # extend an existing table: only new shapes are benchmarked
            to.read_file(table)
        return True
    if not os.path.exists(table):
        return False
    to.enable(True)
    to.tuning_enable(False)
    to.set_filename(table, insert_device_ordinal=False)
    to.read_file(table)
    return True


def flush_tuning():
    """TunableOp writes its table when the process exits; newer torch versions can flush early."""
    import torch

    t = torch.cuda.tunable
    if torch.cuda.is_available() and t.is_enabled() and t.tuning_is_enabled() and hasattr(t, "write_file"):
        t.write_file()
