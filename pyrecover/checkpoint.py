"""Checkpoint API with the reference's signatures (reference pyrecover/checkpoint.py)."""
from pyrecover_amd.ckpt.core import apply_retention, get_latest_checkpoint, wait_all  # noqa: F401
from pyrecover_amd.ckpt.sharded import load_ckpt_distributed, save_ckpt_distributed  # noqa: F401
from pyrecover_amd.ckpt.vanilla import load_ckpt_vanilla, save_ckpt_vanilla, verify_checkpoint  # noqa: F401
