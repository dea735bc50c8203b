#!/usr/bin/env python
"""Drop-in replacement for the reference's ``train.py`` (same flags; see ``--help``).

    python train.py --sequence-length 2048 --batch-size 8 --training-steps 1000 \
        --checkpoint-frequency 100 --verify-checkpoints --timeaware-checkpointing [--distributed]

Launch one process per GPU (``srun`` with SLURM_* env, or ``torchrun --nproc-per-node 8``).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pyrecover_amd.cli import get_args, init_logger  # noqa: E402
from pyrecover_amd.trainer import train  # noqa: E402

if __name__ == "__main__":
    init_logger()
    train(get_args())
