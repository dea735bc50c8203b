"""LR schedule of the reference: linear warmup then constant (reference utils.py:59-81).

Returned as a ``torch.optim.lr_scheduler.LambdaLR`` so its state_dict (``base_lrs``,
``last_epoch``, ``_step_count``, ...) is identical to the reference checkpoint's.
"""
from __future__ import annotations

import functools

from torch.optim.lr_scheduler import LambdaLR


def linear_warmup_constant(warmup_steps: int, current_step: int) -> float:
    if current_step < warmup_steps:
        return float((current_step + 1) / (warmup_steps + 1))
    return 1


def build_lr_scheduler(optimizer, warmup_steps: int) -> LambdaLR:
    return LambdaLR(optimizer, functools.partial(linear_warmup_constant, warmup_steps))
