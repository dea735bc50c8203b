"""Launch-window hooks of the backward pass.

A bandwidth-bound side-stream job (the overlapped AdamW update, :mod:`pyrecover_amd.optim.adamw`)
slows whatever it shares the GPU with. The attention backward offers it a good neighbour: its dK/dV
kernel leaves room on every CU (one 148 KB-LDS block, 2 waves per SIMD) and reads little from HBM,
while the dQ kernel before it fills the register file and the GEMMs around it run at the chip's
power limit. :func:`attention_window` is called with an event that the attention backward records
between its dQ and dK/dV launches; registered jobs enqueue behind that event.

Hooks are scoped to a device: a window on one GPU only releases jobs registered for that GPU.
"""
from __future__ import annotations

import weakref
from typing import Callable, List, Optional, Tuple

_hooks: List[Tuple[Optional[int], weakref.WeakMethod]] = []
_windows = [0]


def add_attention_window_hook(method: Callable, device: Optional[int] = None) -> None:
    """Register a bound method ``fn(event)`` for windows on GPU ``device`` (None: any GPU). Held
    weakly: the owner's lifetime is not extended."""
    _hooks.append((device, weakref.WeakMethod(method)))


def has_hooks() -> bool:
    return any(r() is not None for _, r in _hooks)


def windows_fired() -> int:
    """Number of attention windows offered so far (tests use it to tell which path ran)."""
    return _windows[0]


def attention_window(event, device: Optional[int] = None) -> None:
    _windows[0] += 1
    dead = False
    for dev, ref in _hooks:
        fn = ref()
        if fn is None:
            dead = True
        elif dev is None or device is None or dev == device:
            fn(event)
    if dead:
        _hooks[:] = [(d, r) for d, r in _hooks if r() is not None]
