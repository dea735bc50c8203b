"""Cross-rank replica check: are the DDP replicas still identical?

Data parallelism keeps W copies of the parameters (and, unsharded, of the AdamW moments) that must
stay bitwise equal: every rank applies the same reduced gradient to the same state. Nothing in the
reference notices when they drift (a rank that reduced a different bucket layout, a non-deterministic
kernel, a partial resume): its DDP only broadcasts once at construction (reference
train.py:107-115). Here every rank computes, per buffer, a 64-bit position-weighted hash of the
buffer's words and the fp64 sum of its elements (native kernel ``pra_checksum``, one pass over HBM;
a torch equivalent on the CPU), the ranks all-gather them, and the report says whether they agree.

``bench.py`` runs it after the timed steps (and exits non-zero on a mismatch); ``train.py`` every
``--replica-check-every`` steps (default 10 x ``--logging-frequency``) and at the end. With the
sharded optimizer the moments are per-rank slices and only the parameters are compared.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import _ext

_MASK = (1 << 64) - 1


def _hash_torch(t: torch.Tensor) -> int:
    """sum_i w_i (2 i + 1) mod 2^64 over the 32-bit words of t (the kernel's definition)."""
    flat = t.detach().contiguous().view(-1)
    nbytes = flat.numel() * flat.element_size()
    if nbytes % 4:
        raise ValueError("checksum: buffer size must be a multiple of 4 bytes")
    w = flat.view(torch.uint8).view(torch.int32)
    h = 0
    step = 1 << 22
    for o in range(0, w.numel(), step):
        ww = w[o:o + step].to(torch.int64) & 0xFFFFFFFF
        idx = torch.arange(o, o + ww.numel(), dtype=torch.int64, device=ww.device)
        h = (h + int((ww * (2 * idx + 1)).sum().item())) & _MASK  # int64 products wrap mod 2^64
    return h


def _sum_torch(t: torch.Tensor) -> float:
    flat = t.detach().contiguous().view(-1)
    step = 1 << 24
    return float(sum(float(flat[o:o + step].double().sum()) for o in range(0, flat.numel(), step)))


def buffer_checksum(t: torch.Tensor) -> Tuple[float, int]:
    """(fp64 sum of the elements, 64-bit word hash) of a contiguous buffer."""
    if _ext.hip(t) and (t.numel() * t.element_size()) % 16 == 0 and t.data_ptr() % 16 == 0:
        s, h = _ext.require_for(t).checksum(t.contiguous())
        return float(s.item()), int(h.item()) & _MASK
    return _sum_torch(t), _hash_torch(t)


def _buffers(flat, optimizer) -> Dict[str, torch.Tensor]:
    out = {"params": flat.data}
    sharded = bool(getattr(getattr(flat, "reducer", None), "shard", False))
    if optimizer is not None and not sharded:
        out["exp_avg"] = optimizer.exp_avg
        out["exp_avg_sq"] = optimizer.exp_avg_sq
        if getattr(optimizer, "master", None) is not None:
            out["master_param"] = optimizer.master
    return out


def replica_report(flat, optimizer=None, group=None) -> dict:
    """Collective: checksums of the replicated buffers on every rank and whether they agree.

    Returns ``{"params_identical_across_ranks": bool, "optimizer_identical_across_ranks": bool or None
    (sharded / no optimizer), "mismatched": [buffer names], "checksums": {name: [[sum, hash hex] per
    rank]}}``. A single process reports identical."""
    bufs = _buffers(flat, optimizer)
    mine = {k: buffer_checksum(v) for k, v in bufs.items()}
    world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
    allr: List[Optional[dict]] = [mine]
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, {k: (s, format(h, "016x")) for k, (s, h) in mine.items()}, group=group)
    else:
        allr = [{k: (s, format(h, "016x")) for k, (s, h) in mine.items()}]
    names = list(bufs)
    bad = [k for k in names if any(r[k] != allr[0][k] for r in allr[1:])]
    opt_names = [k for k in names if k != "params"]
    return {
        "params_identical_across_ranks": "params" not in bad,
        "optimizer_identical_across_ranks": (not any(k in bad for k in opt_names)) if opt_names else None,
        "mismatched": bad,
        "checksums": {k: [list(r[k]) for r in allr] for k in names},
    }
