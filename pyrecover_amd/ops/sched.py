"""Launch-window hooks of the backward pass.

A bandwidth-bound side-stream job (the overlapped AdamW update, :mod:`pyrecover_amd.optim.adamw`)
slows whatever it shares the GPU with. The attention backward offers it a good neighbour: its dK/dV
kernel leaves room on every CU (one 148 KB-LDS block, 2 waves per SIMD) and reads little from HBM,
while the dQ kernel before it fills the register file and the GEMMs around it run at the chip's
power limit. :func:`attention_window` is called with an event that the attention backward records
between its dQ and dK/dV launches; registered jobs enqueue behind that event.
"""
from __future__ import annotations

import weakref
from typing import Callable, List

_hooks: List[weakref.WeakMethod] = []


def add_attention_window_hook(method: Callable) -> None:
    """Register a bound method ``fn(event)`` (held weakly: the owner's lifetime is not extended)."""
    _hooks.append(weakref.WeakMethod(method))


def has_hooks() -> bool:
    return any(r() is not None for r in _hooks)


def attention_window(event) -> None:
    dead = False
    for ref in _hooks:
        fn = ref()
        if fn is None:
            dead = True
        else:
            fn(event)
    if dead:
        _hooks[:] = [r for r in _hooks if r() is not None]
