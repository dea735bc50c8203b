#!/usr/bin/env python
"""Prints the parameter count of the reference's default architecture (reference test_model.py),
built on the meta device (no memory)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from pyrecover_amd.config import get_preset  # noqa: E402
from pyrecover_amd.models.llama import Transformer  # noqa: E402


def main(preset: str = "llama3-8b", seq_len: int = 4096):
    with torch.device("meta"):
        model = Transformer(get_preset(preset, seq_len=seq_len))
    n = sum(p.numel() for p in model.parameters())
    print(f"Number of parameters: {n:,}")
    return n


if __name__ == "__main__":
    main(*(sys.argv[1:2] or []))
