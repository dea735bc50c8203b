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
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .flat import FlatParams


class GradReducer:
    """``shard=True`` (``--shard-optimizer``, ZeRO-1 semantics): each bucket is reduce-scattered
    instead of all-reduced -- rank r receives the reduced slice r of it (:meth:`owned`) -- the
    optimizer updates only the owned slices, and :meth:`gather_params` all-gathers the updated
    parameters. Parameters stay replicated; the moments stay allocated full-size (their non-owned
    slices are gathered only for a checkpoint, :meth:`FlatAdamW.gather_state`), so checkpoint formats
    are unchanged. Per bucket the backward moves half the bytes of an all-reduce (the parameter
    all-gather follows the update) and the AdamW update runs on 1/W of the parameters.

    ``sparse_slot`` (``--sparse-embedding-grad``): the index of the embedding's gradient slot. It
    gets a bucket of its own, and instead of a dense all-reduce of the (vocab x dim) gradient, where
    at most B*S rows per rank are non-zero, the ranks exchange (token id, row) pairs
    (:meth:`_sparse_exchange`)."""

    def __init__(self, flat: FlatParams, group=None, bucket_cap_mb: float = 256.0, first_bucket_mb: float = 64.0,
                 backend: str = "rccl", shard: bool = False, sparse_slot: Optional[int] = None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        if backend not in ("rccl", "xgmi"):
            raise ValueError(f"unknown all-reduce backend {backend!r}")
        self.backend = backend if self.world > 1 else "rccl"
        if shard and self.backend == "xgmi":
            raise ValueError("--shard-optimizer runs on RCCL reduce-scatter / all-gather: use --allreduce rccl")
        self.shard = bool(shard) and self.world > 1
        self.sparse_slot = sparse_slot if self.world > 1 else None
        if self.sparse_slot is not None and self.backend == "xgmi":
            raise ValueError("--sparse-embedding-grad runs on RCCL all-gathers: use --allreduce rccl")
        self.hooks = []
        esz = flat.grad.element_size()
        cap = int(bucket_cap_mb * 2 ** 20 / esz)
        first_cap = int(min(first_bucket_mb, bucket_cap_mb) * 2 ** 20 / esz)
        # tail-first greedy packing of slots (slots are in forward order); the sparse embedding slot
        # is a bucket of its own
        buckets: List[List[int]] = []
        cur: List[int] = []
        cur_n = 0
        limit = first_cap  # a smaller first bucket starts communication earlier
        for s in reversed(flat.slots):
            alone = s.index == self.sparse_slot
            if cur and (cur_n + s.numel > limit or alone):
                buckets.append(cur)
                cur, cur_n = [], 0
                limit = cap
            cur.append(s.index)
            cur_n += s.numel
            if alone:
                buckets.append(cur)
                cur, cur_n = [], 0
        if cur:
            buckets.append(cur)
        self.bucket_slots = buckets
        self.ranges = []
        self.padded = self.world > 1 and not getattr(flat, "layout_frozen", False)
        if self.padded:
            # W > 1: every bucket is W equal 64-element-aligned chunks with no remainder
            # (FlatParams.relayout, zero padding after its last group), in both modes, so the
            # sharded optimizer's reduce-scatter chunks a bucket exactly as the all-reduce does and
            # the two modes sum every element in the same order (tests/test_zero1.py)
            self.ranges = flat.relayout(buckets, 64 * self.world)
        elif self.shard:
            raise RuntimeError("--shard-optimizer: build the GradReducer before the optimizer (bucket layout)")
        for b, idxs in enumerate(buckets):
            lo = min(flat.slots[i].offset for i in idxs)
            hi = max(flat.slots[i].offset + flat.slots[i].numel for i in idxs)
            for i in idxs:
                flat.slots[i].bucket = b
            if not self.padded:
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
        # sharded layout: bucket [lo, hi) = W equal chunks of `chunk` elements (a multiple of 64, so
        # every chunk starts 128-B aligned); the shared-tail branches below handle layouts without
        # the relayout's padding (none today)
        self.chunks = []
        for lo, hi in self.ranges:
            m = ((hi - lo) // (64 * self.world)) * 64 * self.world if self.shard else 0
            self.chunks.append(m // self.world if self.shard else 0)
        self.sparse_bucket = flat.slots[self.sparse_slot].bucket if self.sparse_slot is not None else None
        self._emb_scratch = None

    # --- sharded layout ------------------------------------------------------------------
    def owned(self, b: int) -> List[Tuple[int, int]]:
        """Ranges of bucket b whose reduced gradient this rank holds after the reduction, and whose
        parameters it updates: the whole bucket, or (sharded) its chunk plus the shared tail."""
        lo, hi = self.ranges[b]
        if not self.shard:
            return [(lo, hi)]
        c = self.chunks[b]
        out = [(lo + self.rank * c, lo + (self.rank + 1) * c)] if c else []
        if lo + c * self.world < hi:
            out.append((lo + c * self.world, hi))
        return out

    def owned_all(self) -> List[Tuple[int, int]]:
        return [r for b in range(self.num_buckets) for r in self.owned(b)]

    def gather_params(self, b: int, tensors: Sequence[torch.Tensor] = ()):
        """All-gather the owned chunks of bucket b of each tensor laid out like the flat buffer
        (default: the parameters), in place; issued behind the current stream's work. Returns the
        works (empty when not sharded)."""
        if not self.shard or not self.chunks[b]:
            return []
        lo, _ = self.ranges[b]
        c = self.chunks[b]
        works = []
        # `.data`: the in-place gather must not bump the flat buffer's autograd version counter,
        # which every parameter view shares (weights saved for the backward would look modified)
        for t in (tensors or (self.flat.data,)):
            full = t.data[lo:lo + c * self.world]
            works.append(_all_gather_into(full, full[self.rank * c:(self.rank + 1) * c], self.group))
        return works

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
        elif b == self.sparse_bucket:
            work = self._sparse_exchange(b)
            if self.timer is not None:
                self.timer.launched(b, work)
        elif self.shard:
            g, c, W = self.flat.grad, self.chunks[b], self.world
            works = []
            if c:  # in place: rank r's output is chunk r of the input (RCCL's in-place form)
                works.append(_reduce_scatter_into(g[lo + self.rank * c:lo + (self.rank + 1) * c], g[lo:lo + c * W],
                                                  self.group))
            if lo + c * W < hi:
                works.append(dist.all_reduce(g[lo + c * W:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            work = _Works(works)
            if self.timer is not None:
                self.timer.launched(b, work)
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


    # --- sparse embedding-gradient exchange -------------------------------------------------
    def _sparse_exchange(self, b: int):
        """Reduce the embedding gradient as (token id, row) pairs (SURVEY §2.3 K4's 1 GiB tail
        bucket at Llama-3-8B B1: <= B*S of its 131,072 rows are non-zero per rank).

        Each rank sorts its token ids and keeps the first occurrence of each (fixed size n = B*S, the
        rest -1: no host sync), gathers those rows of its dense gradient (the embedding backward's
        deterministic per-id sums), and all-gathers ids and rows (W n (8 + 2 D) bytes instead of an
        all-reduce of V D). Every rank then adds the W contributions of each id in fp32 in rank order
        (one index_add per rank; its indices are unique, so no two adds race) and writes the sum,
        rounded once, into the union's rows; the rows no rank touched stay zero. The result equals the
        rank-ordered fp32 sum of the dense gradients bit for bit. Runs on the current stream (the
        embedding is the last gradient of the backward)."""
        slot = self.flat.slots[self.sparse_slot]
        ids = getattr(slot, "sparse_ids", None)
        if ids is None:
            raise RuntimeError("sparse embedding exchange: the embedding backward recorded no token ids")
        V = slot.params[0].shape[0]
        grad = slot.view.view(V, -1)
        D = grad.shape[1]
        s, _ = torch.sort(ids.reshape(-1))
        first = torch.ones_like(s, dtype=torch.bool)
        first[1:] = s[1:] != s[:-1]
        uid = torch.where(first, s, torch.full_like(s, -1))
        rows = grad.index_select(0, uid.clamp(min=0))  # rows of -1 entries are never read
        n = uid.numel()
        all_ids = torch.empty(self.world * n, dtype=uid.dtype, device=uid.device)
        all_rows = torch.empty(self.world * n, D, dtype=grad.dtype, device=grad.device)
        _all_gather_into(all_ids, uid, self.group).wait()
        _all_gather_into(all_rows, rows, self.group).wait()
        if self._emb_scratch is None or self._emb_scratch.shape != (V + 1, D):
            self._emb_scratch = torch.zeros(V + 1, D, dtype=torch.float32, device=grad.device)
        acc = self._emb_scratch
        ids_w = all_ids.view(self.world, n)
        # -1 entries: accumulate into the spare row V (never read), copy the rank's first id again
        # (its first entry is always valid: the ids are sorted), which writes the same value twice
        add_idx = torch.where(ids_w < 0, torch.full_like(ids_w, V), ids_w)
        copy_idx = torch.where(ids_w < 0, ids_w[:, :1], ids_w).reshape(-1)
        # -0.0 is the identity of IEEE addition: acc ends as g_0 + g_1 + ... + g_{W-1} exactly
        acc.index_fill_(0, add_idx.reshape(-1), -0.0)
        rows_w = all_rows.view(self.world, n, D)
        for r in range(self.world):  # rank order, one fp32 rounding per addition, like the dense sum
            acc.index_add_(0, add_idx[r], rows_w[r].float())
        grad.index_copy_(0, copy_idx, acc.index_select(0, copy_idx).to(grad.dtype))
        slot.sparse_ids = None
        return None


def _gloo_cuda(t: torch.Tensor, group) -> bool:
    # gloo with device tensors is the one-GPU multi-rank rehearsal (RCCL refuses two ranks on one
    # GPU); there the tensor collectives run through the forms gloo implements for device tensors
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _reduce_scatter_into(out: torch.Tensor, inp: torch.Tensor, group):
    """out (chunk `rank` of inp, possibly aliasing it) = SUM over ranks of that chunk."""
    if _gloo_cuda(inp, group):
        tmp = inp.clone()
        dist.all_reduce(tmp, group=group)  # gloo: the same per-element order as its reduce-scatter
        r, c = dist.get_rank(group), out.numel()
        out.copy_(tmp[r * c:(r + 1) * c])
        return _Works([])
    return dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group, async_op=True)


def _all_gather_into(full: torch.Tensor, part: torch.Tensor, group):
    """full = concat over ranks of `part` (part may alias its own chunk of full)."""
    if _gloo_cuda(full, group):
        parts = [torch.empty_like(part) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, part.contiguous(), group=group)
        full.copy_(torch.cat(parts))
        return _Works([])
    return dist.all_gather_into_tensor(full, part, group=group, async_op=True)


class _Works:
    """Several collectives of one bucket waited for together (reduce-scatter + tail all-reduce)."""

    __slots__ = ("works",)

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()

    def is_completed(self):
        return all(w.is_completed() for w in self.works)


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
