"""PyRecover API (reference pyrecover/__init__.py), implemented on the pyrecover_amd engine.

All five names the reference exports are real here (the reference's resubmit/timelimit modules
were missing)."""

__version__ = "0.1.0"

from .checkpoint import load_ckpt_vanilla, save_ckpt_vanilla  # noqa: F401
from .resubmit import setup_resubmission  # noqa: F401
from .timelimit import get_remaining_time, monitor_timelimit  # noqa: F401

__all__ = [
    "save_ckpt_vanilla",
    "load_ckpt_vanilla",
    "monitor_timelimit",
    "get_remaining_time",
    "setup_resubmission",
]
