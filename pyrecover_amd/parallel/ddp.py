"""Bucketed gradient all-reduce over the flat gradient buffer (replaces torch DDP, reference
train.py:107-115 and its Reducer).

* Buckets are contiguous slices of the flat gradient buffer built tail-first (the order in which
  gradients become ready during backward), aligned to fusion-group boundaries, so each bucket is
  all-reduced IN PLACE with one RCCL call: no copy-in / copy-out, no per-parameter views.
* A bucket is launched (``async_op=True``) from the backward thread the moment its last gradient
  slot is written; RCCL runs it on its own stream, overlapped with the rest of backward, and the
  compute stream only waits on it in :meth:`GradReducer.finish` (GPU-side wait, no host sync).
* Bucket size defaults to 256 MiB: on MI355X each GPU has 7 xGMI links (~153 GB/s each), a ring
  collective moves bucket/8 per link-step, and chunks below ~4-8 MiB per link lose efficiency;
  large buckets also keep the per-step collective count low (~55 for a 7B model instead of the
  ~162 25-MiB buckets of torch DDP's default).
* The gradient is SUM-reduced; the 1/world_size average is folded into the optimizer kernel
  (``FlatAdamW.grad_scale``), so there is no separate scaling pass.
* Deterministic: identical bucket order/boundaries on every rank and every step.
* ``backend="xgmi"`` swaps RCCL for the direct per-link all-reduce of
  :mod:`pyrecover_amd.parallel.xgmi` (same buckets, same hooks).
* With ``world_size == 1`` (or no process group) the same bucket machinery runs without
  communication, so bucket hooks (the overlapped optimizer) work identically on one GPU.
* Bucket hooks ``fn(bucket, lo, hi, work)`` run right after a bucket is launched; the
  overlapped AdamW (:meth:`pyrecover_amd.optim.adamw.FlatAdamW.enable_overlap`) uses them to
  update each bucket's parameters on a side stream while backward continues.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .flat import FlatParams


class GradReducer:
    def __init__(self, flat: FlatParams, group=None, bucket_cap_mb: float = 256.0, first_bucket_mb: float = 64.0,
                 backend: str = "rccl"):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        if backend not in ("rccl", "xgmi"):
            raise ValueError(f"unknown all-reduce backend {backend!r}")
        self.backend = backend if self.world > 1 else "rccl"
        self.hooks = []
        esz = flat.grad.element_size()
        cap = int(bucket_cap_mb * 2 ** 20 / esz)
        first_cap = int(min(first_bucket_mb, bucket_cap_mb) * 2 ** 20 / esz)
        # tail-first greedy packing of slots (slots are in forward order)
        buckets: List[List[int]] = []
        cur: List[int] = []
        cur_n = 0
        limit = first_cap  # a smaller first bucket starts communication earlier
        for s in reversed(flat.slots):
            if cur and cur_n + s.numel > limit:
                buckets.append(cur)
                cur, cur_n = [], 0
                limit = cap
            cur.append(s.index)
            cur_n += s.numel
        if cur:
            buckets.append(cur)
        self.bucket_slots = buckets
        self.ranges = []
        for b, idxs in enumerate(buckets):
            lo = min(flat.slots[i].offset for i in idxs)
            hi = max(flat.slots[i].offset + flat.slots[i].numel for i in idxs)
            for i in idxs:
                flat.slots[i].bucket = b
            self.ranges.append((lo, hi))
        # extend the last bucket to the end of the buffer / first to 0 so padding is covered
        self.counts = [len(b) for b in buckets]
        self.pending = list(self.counts)
        self.works: List[Optional[object]] = [None] * len(buckets)
        self.next_to_launch = 0
        self.enabled = True
        flat.reducer = self
        self.timer: Optional["CommTimer"] = None
        # diagnostic (tools/queue_probe.py): issue the RCCL all-reduce even in a 1-rank group, so a
        # 1-GPU trace shows the collective's stream beside compute
        self.force_collective = (os.environ.get("PYRECOVER_FORCE_ALLREDUCE") == "1" and dist.is_available()
                                 and dist.is_initialized())
        self.xgmi = None
        if self.backend == "xgmi":
            from .xgmi import XgmiAllReduce

            self.xgmi = XgmiAllReduce(flat, self.ranges, group)

    @property
    def num_buckets(self) -> int:
        return len(self.bucket_slots)

    def bucket_bytes(self) -> List[int]:
        e = self.flat.grad.element_size()
        return [(hi - lo) * e for lo, hi in self.ranges]

    def reset(self):
        self.pending = list(self.counts)
        self.works = [None] * len(self.counts)
        self.next_to_launch = 0

    def mark_ready(self, slot):
        if not self.enabled:
            return
        b = slot.bucket
        self.pending[b] -= 1
        # launch strictly in bucket order so every rank issues the same collective sequence
        while self.next_to_launch < len(self.pending) and self.pending[self.next_to_launch] == 0:
            self._launch(self.next_to_launch)
            self.next_to_launch += 1

    def _launch(self, b: int):
        lo, hi = self.ranges[b]
        work = None
        if self.timer is not None:
            self.timer.ready(b)
        if self.xgmi is not None:
            work = self.xgmi.launch(b)
        elif self.world > 1 or self.force_collective:
            work = dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if self.timer is not None:
                self.timer.launched(b, work)
        self.works[b] = work
        for h in self.hooks:
            h(b, lo, hi, work)

    def finish(self):
        """Launch any bucket whose slots were not all produced (unused params), then make the
        current stream wait for every collective."""
        if not self.enabled:
            return
        while self.next_to_launch < len(self.pending):
            self._launch(self.next_to_launch)
            self.next_to_launch += 1
        if self.timer is not None:
            self.timer.before_finish(self.works)
        for w in self.works:
            if w is not None:
                w.wait()
        if self.timer is not None:
            self.timer.after_finish()
        self.works = [None] * len(self.counts)
        if self.xgmi is not None:
            self.xgmi.end_step()

    def enable_comm_timing(self) -> "CommTimer":
        """Per-step, per-bucket collective timing (bench.py for W > 1)."""
        if self.timer is None:
            self.timer = CommTimer(self)
        return self.timer


def comm_env() -> Dict[str, str]:
    """The RCCL/NCCL tuning environment in effect (NCCL_* / RCCL_* / HSA_* / PYRECOVER_RCCL_*)."""
    keep = ("NCCL_", "RCCL_", "TORCH_NCCL_", "HSA_ENABLE_IPC", "PYRECOVER_RCCL", "GPU_MAX_HW_QUEUES")
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith(keep)}


class CommTimer:
    """Timing of the gradient collectives of each step, so an N-GPU result is diagnosable.

    GPU: events only, no host sync inside the step.
      * ``ready[b]``: recorded on the compute stream when bucket b is launched (its gradients are
        enqueued);
      * ``end[b]``: recorded on a side stream made to wait for bucket b's collective (RCCL: right
        at launch; xGMI: at finish, since its ``wait`` blocks the host until enqueued);
      * ``bwd_end`` / ``fin``: the compute stream right before / after :meth:`GradReducer.finish`
        waits for the collectives.
      Collectives of one process group run in order on one stream, so bucket b is busy from
      max(ready[b], end[b-1]) to end[b]; ``exposed_comm_ms`` = fin - bwd_end is the time the
      compute stream idles on communication after the backward's last kernel.
    CPU (gloo rehearsal): host clocks; each bucket is waited for as soon as it is launched.
    """

    def __init__(self, reducer: GradReducer):
        self.r = reducer
        self.cuda = reducer.flat.grad.is_cuda
        self.nb = reducer.num_buckets
        self.bytes = reducer.bucket_bytes()
        self.steps: List[dict] = []
        self._cur = None
        self.active = False
        if self.cuda:
            self.side = torch.cuda.Stream(device=reducer.flat.grad.device)

    def _mark(self, stream=None):
        if not self.cuda:
            return time.perf_counter()
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream) if stream is not None else e.record()
        return e

    def begin_step(self):
        self.active = True
        self._cur = {"t0": self._mark(), "ready": [None] * self.nb, "end": [None] * self.nb}

    def ready(self, b):
        if self.active:
            self._cur["ready"][b] = self._mark()

    def launched(self, b, work):
        if not self.active or work is None:
            return
        if self.cuda:
            with torch.cuda.stream(self.side):
                work.wait()
                self._cur["end"][b] = self._mark(self.side)
        else:  # CPU: the overlapped optimizer waits for the bucket right away anyway
            work.wait()
            self._cur["end"][b] = self._mark()

    def before_finish(self, works):
        if not self.active:
            return
        c = self._cur
        c["bwd_end"] = self._mark()
        if self.cuda:
            with torch.cuda.stream(self.side):
                for b, w in enumerate(works):
                    if c["end"][b] is None and w is not None:
                        w.wait()
                        c["end"][b] = self._mark(self.side)
        else:
            for b, w in enumerate(works):
                if c["end"][b] is None and w is not None:
                    w.wait()
                    c["end"][b] = self._mark()

    def after_finish(self):
        if not self.active:
            return
        self._cur["fin"] = self._mark()
        self.steps.append(self._cur)
        self._cur = None
        self.active = False

    def _ms(self, a, b) -> float:
        return a.elapsed_time(b) if self.cuda else 1000.0 * (b - a)

    def summary(self, world: int) -> dict:
        """Mean over the timed steps (call after a device synchronize)."""
        if not self.steps:
            return {}
        n = len(self.steps)
        busy = [0.0] * self.nb
        exposed = 0.0
        for c in self.steps:
            t = lambda e: self._ms(c["t0"], e)  # noqa: E731
            exposed += self._ms(c["bwd_end"], c["fin"])
            prev_end = None
            for b in range(self.nb):
                if c["end"][b] is None or c["ready"][b] is None:
                    continue
                start = t(c["ready"][b]) if prev_end is None else max(t(c["ready"][b]), prev_end)
                end = t(c["end"][b])
                busy[b] += max(end - start, 0.0)
                prev_end = end
        busy = [x / n for x in busy]
        algbw = [(by / 1e9) / (ms / 1e3) if ms > 0 else None for by, ms in zip(self.bytes, busy)]
        f = 2.0 * (world - 1) / world
        tot_ms = sum(busy)
        tot_b = sum(self.bytes)
        return {
            "exposed_comm_ms": round(exposed / n, 3),
            "allreduce_busy_ms": round(tot_ms, 3),
            "allreduce_gib": round(tot_b / 2**30, 3),
            "allreduce_busbw_gbps": round(f * (tot_b / 1e9) / (tot_ms / 1e3), 4) if tot_ms > 0 else None,
            "buckets": [{"mib": round(by / 2**20, 1), "ms": round(ms, 3),
                         "algbw_gbps": round(a, 1) if a else None, "busbw_gbps": round(f * a, 1) if a else None}
                        for by, ms, a in zip(self.bytes, busy, algbw)],
            "timing_source": "hip events" if self.cuda else "host clock (gloo CPU rehearsal)",
        }


def broadcast_flat(flat: FlatParams, src: int = 0, group=None, chunk_mb: int = 1024):
    """Replicate rank ``src``'s parameters (reference DDP ctor broadcast)."""
    n = flat.numel
    step = max(1, int(chunk_mb * 2 ** 20 / flat.data.element_size()))
    for o in range(0, n, step):
        dist.broadcast(flat.data[o:o + step], src=src, group=group)
    flat.refresh_transposed()
