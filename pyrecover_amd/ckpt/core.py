"""Checkpoint engine front-end: state collection, staging, async jobs, latest/retention.

Everything here is format-agnostic; :mod:`.vanilla` and :mod:`.sharded` build on it.

Staging: all tensors of a checkpoint state are mapped to contiguous byte regions of their
storages (the flat parameter / Adam buffers collapse into a few large regions), copied by the
C++ engine into a reusable pinned host pool (device: hipMemcpyAsync on a low-priority stream;
CPU: parallel memcpy) and replaced in the state by CPU tensors aliasing the pool. The archive
writer thread then streams them to disk while training continues; :meth:`Checkpointer.fence`
makes the compute stream wait for the snapshot before the optimizer mutates parameters again.
"""
from __future__ import annotations

import atexit
import logging
import os
import random
import re
import shutil
import threading
import time
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from .. import _ext
from .serialization import host_view

logger = logging.getLogger("pyrecover")

_MERGE_GAP = 4096  # bytes: merge staging regions separated by small alignment gaps


# ------------------------------------------------------------------------------------------
def unwrap(model):
    m = model
    while True:
        if hasattr(m, "module") and isinstance(getattr(m, "module"), torch.nn.Module):
            m = m.module
        elif hasattr(m, "_orig_mod") and isinstance(getattr(m, "_orig_mod"), torch.nn.Module):
            m = m._orig_mod
        else:
            return m


_PREFIX_RE = re.compile(r"^(module\.|_orig_mod\.)+")


def strip_prefixes(sd: Dict[str, Any]) -> Dict[str, Any]:
    """World-size / compile agnostic keys."""
    return {_PREFIX_RE.sub("", k): v for k, v in sd.items()}


def capture_rng_state() -> Dict[str, Any]:
    st = {"torch_cpu": torch.get_rng_state(), "python": random.getstate()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["torch_cuda"] = torch.cuda.get_rng_state_all()
    return st


def restore_rng_state(st: Dict[str, Any]):
    if not st:
        return
    if "torch_cpu" in st:
        torch.set_rng_state(st["torch_cpu"])
    if "python" in st:
        v = st["python"]
        random.setstate((v[0], tuple(v[1]), v[2]))
    if "torch_cuda" in st and torch.cuda.is_available():
        states = st["torch_cuda"]
        if len(states) == torch.cuda.device_count():
            torch.cuda.set_rng_state_all(states)
    if "torch_cuda_device" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["torch_cuda_device"])  # this rank's own device


def capture_rank_rng_state() -> Dict[str, Any]:
    """This rank's RNG streams: CPU, python and the generator of the rank's own device."""
    st = {"torch_cpu": torch.get_rng_state(), "python": random.getstate()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["torch_cuda_device"] = torch.cuda.get_rng_state()
    return st


def gather_rng_states() -> Optional[List[Dict[str, Any]]]:
    """Collective: every rank's :func:`capture_rank_rng_state`, indexed by rank (None without a
    multi-rank process group). Checkpoints store the list as ``pyrecover_state.rng_per_rank`` so
    a resumed DDP job restores each rank's own streams, not rank 0's."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return None
    w = torch.distributed.get_world_size()
    if w <= 1:
        return None
    out: List[Any] = [None] * w
    torch.distributed.all_gather_object(out, capture_rank_rng_state())
    return out


def restore_rng_from(ps: Optional[Dict[str, Any]]):
    """Restore this rank's RNG from a checkpoint's ``pyrecover_state``: its own entry of
    ``rng_per_rank`` when the world size matches, else the saving process's ``rng``."""
    ps = ps or {}
    warn_reduction_change(ps)
    per = ps.get("rng_per_rank")
    if per:
        per = [per[k] for k in sorted(per, key=int)] if isinstance(per, dict) else list(per)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
    else:
        rank, world = 0, 1
    if per and len(per) == world:
        restore_rng_state(per[rank])
    else:
        restore_rng_state(ps.get("rng"))


def warn_reduction_change(ps: Optional[Dict[str, Any]]) -> List[str]:
    """Warn when the checkpoint was written under different gradient-reduction settings (world size,
    backend, RCCL algorithm / protocol / channels): the resumed run is then not guaranteed to be
    bit-identical to an uninterrupted one. PYRECOVER_RCCL_DETERMINISTIC=1 pins them."""
    from ..parallel import dist as _dist

    diffs = _dist.compare_rccl_order((ps or {}).get("reduction"))
    if diffs and _dist.is_rank0():
        logger.warning("checkpoint was written with different gradient-reduction settings; the resumed run "
                       "may not be bit-identical to an uninterrupted one: " + "; ".join(diffs))
    return diffs


def peek_reduction(path: str, exp_dir: Optional[Path] = None, distributed: bool = False) -> Optional[Dict[str, Any]]:
    """The gradient-reduction settings a checkpoint was written with (``pyrecover_state.reduction``),
    read without loading its tensors (``latest`` resolves as the loaders do); None if there is none."""
    try:
        if path == "latest":
            path = get_latest_checkpoint(str(exp_dir), distributed) if exp_dir is not None else None
            if path is None:
                return None
        p = Path(path)
        if p.is_dir():
            from .sharded import read_metadata, read_sharded_state

            keep = [i.fqn for i in read_metadata(p).storage_data if i.fqn.startswith("pyrecover_state.reduction")]
            skip = {i.fqn for i in read_metadata(p).storage_data} - set(keep)
            st = read_sharded_state(str(p), skip=skip)
        else:
            # mmap: the tensors' bytes are not read
            st = torch.load(str(p), map_location="cpu", mmap=True, weights_only=True)
        return ((st or {}).get("pyrecover_state") or {}).get("reduction")
    except Exception as e:  # noqa: BLE001 - an unreadable checkpoint fails later, in the loader
        logger.warning(f"could not read the reduction settings of {path}: {e}")
        return None


def prepare_optimizer_state(optimizer):
    """Collective, on every rank before a save: the sharded optimizer all-gathers its moments so the
    checkpoint holds the full state (a no-op for the replicated optimizer)."""
    fn = getattr(optimizer, "gather_state", None)
    if fn is not None:
        fn()


def build_state(model, optimizer, lr_scheduler=None, sampler=None, step: int = 0, epoch: Optional[int] = None,
                extra: Optional[Dict[str, Any]] = None,
                rng_per_rank: Optional[List[Dict[str, Any]]] = None) -> Dict[str, Any]:
    """The reference's vanilla checkpoint dict (reference pyrecover/checkpoint.py:60-73) plus a
    ``pyrecover_state`` entry (RNG, sampler cursor, run metadata) that reference loaders ignore."""
    m = unwrap(model)
    state: Dict[str, Any] = {
        "epoch": epoch,
        "step": step,
        "model": strip_prefixes(m.state_dict()),
        "optimizer": optimizer.state_dict(),
    }
    if lr_scheduler is not None:
        state["lr_scheduler"] = lr_scheduler.state_dict()
    if sampler is not None and hasattr(sampler, "set_state"):
        state["sampler_state"] = sampler.state_dict()
    from ..parallel import dist as _dist

    ps = {"format": "pyrecover_amd/1", "rng": capture_rng_state(), "saved_at": time.time(),
          "reduction": _dist.rccl_order_settings()}
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        ps["world_size"] = torch.distributed.get_world_size()
    if rng_per_rank is not None:
        ps["rng_per_rank"] = rng_per_rank
    if extra:
        ps.update(extra)
    state["pyrecover_state"] = ps
    return state


# ------------------------------------------------------------------------------------------
def _walk(obj, fn):
    """Rebuild a nested dict/list/tuple structure with fn applied to tensor leaves."""
    if isinstance(obj, torch.Tensor):
        return fn(obj)
    if isinstance(obj, dict):
        return obj.__class__((k, _walk(v, fn)) for k, v in obj.items())
    if isinstance(obj, list):
        return [_walk(v, fn) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_walk(v, fn) for v in obj)
    return obj


def _tensors(obj, out: List[torch.Tensor]):
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, dict):
        for v in obj.values():
            _tensors(v, out)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _tensors(v, out)
    return out


class Checkpointer:
    """Per-device staging pool + background writer (one in-flight archive per device)."""

    _instances: Dict[int, "Checkpointer"] = {}

    @classmethod
    def get(cls, device: torch.device) -> "Checkpointer":
        idx = device.index if device.type == "cuda" else -1
        if device.type == "cuda" and idx is None:
            idx = torch.cuda.current_device()
        if idx not in cls._instances:
            cls._instances[idx] = Checkpointer(idx)
        return cls._instances[idx]

    def __init__(self, device_index: int):
        self.device_index = device_index
        self.engine = _ext.native().CkptEngine(device_index)
        self.pending: Optional["Job"] = None
        self.staged = False
        self._prewarm: Optional[threading.Thread] = None
        self._hbm: Optional[torch.Tensor] = None

    def prewarm(self, nbytes: int, background: bool = True):
        """Allocate the pinned staging pool ahead of the first checkpoint. Prefer
        ``background=False`` before training starts: hipHostMalloc updates the GPU page tables,
        which serializes behind running kernels (a background allocation overlapping the first
        training steps stalled them for minutes on MI355X), while on an idle GPU it takes ~0.2 s/GB."""
        if self._prewarm is not None or nbytes <= self.engine.pool_size():
            return
        if not background:
            self.engine.reserve(int(nbytes))
            return
        self._prewarm = threading.Thread(target=self.engine.reserve, args=(int(nbytes),), daemon=True,
                                         name="pyrecover-ckpt-prewarm")
        self._prewarm.start()

    def _join_prewarm(self):
        if self._prewarm is not None:
            self._prewarm.join()
            self._prewarm = None

    # -- staging -------------------------------------------------------------------------
    def stage(self, obj):
        """Snapshot every tensor of ``obj`` on this checkpointer's device into the pinned pool;
        return ``obj`` rebuilt with CPU tensors aliasing the pool (other tensors are cloned)."""
        self._join_prewarm()
        self.wait()  # pool reuse: the previous archive must be on disk
        dev_is_cuda = self.device_index >= 0
        ts = _tensors(obj, [])
        spans: List[Tuple[int, int, int]] = []  # (ptr, nbytes, storage base)
        for t in ts:
            on_dev = t.is_cuda if dev_is_cuda else (not t.is_cuda)
            if not on_dev or t.numel() == 0:
                continue
            if not t.is_contiguous():
                raise ValueError("checkpoint tensors must be contiguous")
            spans.append((t.data_ptr(), t.numel() * t.element_size(), t.untyped_storage().data_ptr()))
        spans.sort()
        regions: List[List[int]] = []  # [ptr, nbytes, storage base]
        for p, n, sb in spans:
            # merge only inside ONE storage: a gap between two allocations may be unmapped memory
            if regions and regions[-1][2] == sb and p <= regions[-1][0] + regions[-1][1] + _MERGE_GAP:
                regions[-1][1] = max(regions[-1][1], p + n - regions[-1][0])
            else:
                regions.append([p, n, sb])
        total = sum(r[1] for r in regions) + 64 * len(regions)
        if total > self.engine.pool_size():
            self.engine.reserve(int(total * 1.05) + (1 << 20))
        hbm = self._hbm_buffer(total) if (dev_is_cuda and regions) else None
        offs = (self.engine.stage([(r[0], r[1]) for r in regions], hbm.data_ptr() if hbm is not None else 0,
                                  hbm.numel() if hbm is not None else 0) if regions else [])
        base = self.engine.pool_ptr()
        starts = [r[0] for r in regions]
        import bisect

        def to_host(t: torch.Tensor):
            on_dev = t.is_cuda if dev_is_cuda else (not t.is_cuda)
            if not on_dev or t.numel() == 0:
                return t.detach().to("cpu", copy=True)
            i = bisect.bisect_right(starts, t.data_ptr()) - 1
            host = base + offs[i] + (t.data_ptr() - starts[i])
            return host_view(host, t.numel() * t.element_size(), t.dtype, tuple(t.shape))

        self.staged = True
        return _walk(obj, to_host)

    def _hbm_buffer(self, nbytes: int) -> Optional[torch.Tensor]:
        """Device-side bounce buffer of the two-hop snapshot: the live buffers are
        copied into it at HBM bandwidth, the next update is fenced only on that copy, and the D2H
        into the pinned pool drains from it. Kept across saves (one allocation); None -- direct
        D2H as before -- when PYRECOVER_CKPT_HBM=0 or free HBM would drop below the reserve
        (PYRECOVER_CKPT_HBM_RESERVE_GB, default 8) after allocating it."""
        if os.environ.get("PYRECOVER_CKPT_HBM", "1") == "0":
            return None
        if self._hbm is not None and self._hbm.numel() >= nbytes:
            return self._hbm
        dev = torch.device("cuda", self.device_index)
        self._hbm = None  # the previous snapshot was fully drained (stage() waited for the writer)
        free, _ = torch.cuda.mem_get_info(dev)
        reserve = float(os.environ.get("PYRECOVER_CKPT_HBM_RESERVE_GB", "8")) * 2**30
        if free - nbytes < reserve:
            logger.info(f"checkpoint snapshot: {nbytes / 2**30:.1f} GiB HBM bounce buffer does not fit "
                        f"({free / 2**30:.1f} GiB free): direct D2H, the next update waits for it")
            return None
        try:
            self._hbm = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        except torch.OutOfMemoryError:
            logger.info(f"checkpoint snapshot: {nbytes / 2**30:.1f} GiB HBM bounce buffer allocation failed: "
                        f"direct D2H, the next update waits for it")
            return None
        return self._hbm

    def release_hbm(self):
        """Free the bounce buffer (OOM recovery: training allocations take precedence over the
        two-hop snapshot; the next save re-checks the free memory)."""
        self.wait()
        self._hbm = None

    def fence(self):
        """Make the current compute stream wait (GPU-side) for the in-flight snapshot: with the HBM
        bounce buffer, for its device-to-device copy only."""
        if self.staged and self.device_index >= 0:
            self.engine.fence()

    def sync_stage(self):
        if self.staged:
            self.engine.sync_stage()

    # -- writing -------------------------------------------------------------------------
    def write(self, path: str, items, md5: bool, fsync: bool, keepalive, on_done: Optional[Callable] = None,
              defer_md5: bool = False) -> "Job":
        """defer_md5: the job completes once the archive and ``.md5parts`` are durable; the
        reference's whole-file ``.md5`` (serial MD5) is computed in the background by re-reading
        the file (no staging memory held) -- :func:`flush_all` (also at exit) waits for it."""
        self.wait()
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        self.engine.write_items(str(path), items, md5, fsync, defer_md5)
        self.pending = Job(self, str(path), keepalive, on_done, started=time.perf_counter())
        _maybe_inject_fault("during_write", path)
        return self.pending

    def busy(self) -> bool:
        return self.engine.busy()

    def wait(self) -> Optional[Dict[str, Any]]:
        job, self.pending = self.pending, None
        if job is None:
            return None
        return job.wait()

    def poll(self):
        """Collect a finished background write without blocking (records its duration)."""
        if self.pending is not None and not self.engine.busy():
            self.wait()

    def flush(self):
        """Wait for the in-flight write and any deferred whole-file ``.md5`` digest."""
        self.wait()
        err = self.engine.flush()
        if err:
            raise RuntimeError(f"deferred checkpoint md5 failed: {err}")


# Background-write durations feed the time-aware stop: the FINAL checkpoint is written
# synchronously (and first drains any in-flight write), so the stop threshold must budget the
# full write time, not the ~ms an async save stalls training.
WRITE_STATS: Dict[str, Any] = {"max_seconds": 0.0, "min_write_bps": 0.0, "min_inline_bps": 0.0}
_RATE_MIN_BYTES = 64 << 20  # smaller jobs are overhead-dominated: their rates are not recorded


def _record_rates(res: Dict[str, Any]):
    """Per-byte rates of a completed archive job (slowest seen): plain writes, and writes that
    computed the whole-file MD5 inline (their time is max(write, serial MD5))."""
    nb = int(res.get("bytes", 0))
    sec = float(res.get("write_seconds", 0.0)) + float(res.get("fsync_seconds", 0.0))
    if nb < _RATE_MIN_BYTES or sec <= 0:
        return
    key = "min_inline_bps" if (res.get("md5") and not res.get("md5_deferred")) else "min_write_bps"
    bps = nb / sec
    WRITE_STATS[key] = bps if WRITE_STATS[key] <= 0 else min(WRITE_STATS[key], bps)


@dataclass
class Job:
    ckpt: Checkpointer
    path: str
    keepalive: Any
    on_done: Optional[Callable]
    result: Optional[Dict[str, Any]] = None
    started: float = 0.0

    def wait(self) -> Dict[str, Any]:
        if self.result is None:
            self.result = self.ckpt.engine.wait()
            self.keepalive = None
            if not self.result["ok"]:
                raise RuntimeError(f"checkpoint write to {self.path} failed: {self.result['error']}")
            WRITE_STATS["max_seconds"] = max(WRITE_STATS["max_seconds"], float(self.result.get("seconds", 0.0)))
            _record_rates(self.result)
            WRITE_STATS["last"] = {k: v for k, v in self.result.items() if k not in ("items", "records", "seg_md5")}
            WRITE_STATS["jobs"] = WRITE_STATS.get("jobs", 0) + 1
            if self.on_done is not None:
                self.on_done(self.result)
        return self.result


def poll_all():
    for c in Checkpointer._instances.values():
        c.poll()


def max_write_seconds() -> float:
    """Longest completed background archive write (0 if none yet)."""
    return WRITE_STATS["max_seconds"]


class SaveCostModel:
    """Predicted wall-clock of the time-aware FINAL save, and of the drain of an in-flight async
    save, from bytes and measured rates.

    The reference budgets a running maximum of completed save times (train.py:298-307), which
    knows nothing until a save has completed: a job whose first save is the final one gets the
    10 s prior whatever the model size. Here the final save costs

        overhead + bytes / d2h + max(bytes / write rate, bytes / MD5 rate  [inline .md5 only])

    with rates from a startup probe (:meth:`probe`: the archive writer's parallel O_DIRECT path
    into the checkpoint directory, and the single-stream MD5 of the reference's whole-file
    ``.md5``) until real saves report their own (slowest seen; a save that computed its digest
    inline bounds the whole final save directly). ``bytes`` is what THIS rank writes (the whole
    state for vanilla, ~1/W of it for sharded)."""

    OVERHEAD_S = 2.0  # pickling, metadata, barriers, rename + sidecars

    def __init__(self, state_bytes: int, inline_md5: bool, d2h_gbps: Optional[float] = None):
        self.state_bytes = int(state_bytes)
        self.inline_md5 = bool(inline_md5)
        if d2h_gbps is None:
            d2h_gbps = float(os.environ.get("PYRECOVER_D2H_GBPS", "20"))
        self.d2h_bps = d2h_gbps * 1e9
        self.probe_write_bps = 0.0
        self.probe_md5_bps = 0.0

    def probe(self, directory, write_bytes: Optional[int] = None, md5_bytes: int = 256 << 20):
        """Measure the write rate into ``directory`` (a probe file of ``write_bytes``, default
        clamp(state, 256 MiB, 2 GiB), removed afterwards) and the serial MD5 rate."""
        n = _ext.native()
        if write_bytes is None:
            write_bytes = int(os.environ.get("PYRECOVER_CKPT_PROBE_BYTES", "0")) or \
                min(max(self.state_bytes, 256 << 20), 2 << 30)
        os.makedirs(str(directory), exist_ok=True)
        import socket

        path = os.path.join(str(directory), f".pyrecover_write_probe.{socket.gethostname()}.{os.getpid()}.tmp")
        self.probe_write_bps = float(n.write_probe_bps(path, int(write_bytes), int(n.CKPT_WRITERS), True))
        if self.inline_md5:
            self.probe_md5_bps = float(n.md5_probe_bps(int(md5_bytes)))
        return self

    @property
    def write_bps(self) -> float:
        return WRITE_STATS["min_write_bps"] or self.probe_write_bps

    @property
    def md5_bps(self) -> float:
        rates = [r for r in [self.probe_md5_bps] + [c.engine.md5_min_bps() for c in Checkpointer._instances.values()]
                 if r > 0]
        return min(rates) if rates else 0.0

    @staticmethod
    def _t(nbytes: float, bps: float) -> float:
        return nbytes / bps if bps > 0 else 0.0

    def final_seconds(self, nbytes: Optional[int] = None) -> float:
        nb = self.state_bytes if nbytes is None else int(nbytes)
        body = self._t(nb, self.write_bps)
        if self.inline_md5:
            body = max(body, self._t(nb, self.md5_bps), self._t(nb, WRITE_STATS["min_inline_bps"]))
        return self.OVERHEAD_S + self._t(nb, self.d2h_bps) + body

    def drain_seconds(self, final_budget: float) -> float:
        """Extra seconds before the job can exit, beyond ``final_budget`` for the final save, that
        in-flight work adds: the final save starts only once the in-flight archive is written
        (the pinned pool is reused), and deferred whole-file digests (of the in-flight save, or
        queued) must finish before exit. Estimated from the bytes still to write / hash."""
        write_rem, digest_end = 0.0, 0.0
        for c in Checkpointer._instances.values():
            j = c.pending
            busy = j is not None and j.result is None and c.engine.busy()
            total, written, hashed, mode = c.engine.progress() if busy else (0, 0, 0, 0)
            w = self._t(max(total - written, 0), self.write_bps)
            if mode == 1:  # inline whole-file digest of the in-flight save
                w = max(w, self._t(max(total - hashed, 0), self.md5_bps))
            write_rem = max(write_rem, w)
            pending = c.engine.md5_pending_bytes() + (total if mode == 2 else 0)
            d = self._t(pending, self.md5_bps)
            digest_end = max(digest_end, (w if mode == 2 else 0.0) + d)
        return max(write_rem + final_budget, digest_end) - final_budget


# vanilla checkpoints whose whole-file .md5 this process left to a deferred background digest
DEFERRED_MD5_PATHS: set = set()


def drop_unverified(base: Path, keep: str, only: Optional[set] = None) -> List[str]:
    """After a time-aware stop whose final checkpoint carries its ``.md5``: remove older vanilla
    checkpoints whose deferred digest THIS process queued and abandoned at the wall-clock limit (no
    ``.md5``), so with ``--verify-checkpoints`` every checkpoint this job wrote verifies with the
    reference's loader (reference pyrecover/checkpoint.py:157-175). Checkpoints of earlier jobs
    (e.g. written without --verify-checkpoints) are never touched. ``only`` defaults to
    :data:`DEFERRED_MD5_PATHS`. Returns the removed paths."""
    removed = []
    only = DEFERRED_MD5_PATHS if only is None else only
    keep_step = ckpt_step(Path(keep))
    for f in Path(base).glob("ckpt_*.pt"):
        if str(f) not in only:
            continue
        if str(f) == str(keep) or ckpt_step(f) >= keep_step or Path(str(f) + ".md5").exists():
            continue
        try:
            f.unlink()
            for side in (".md5parts",):
                sp = Path(str(f) + side)
                if sp.exists():
                    sp.unlink()
            removed.append(str(f))
        except FileNotFoundError:
            pass
    return removed


def flush_all(deadline: Optional[float] = None) -> bool:
    """wait_all() plus the deferred whole-file ``.md5`` digests (their sidecars exist afterwards).
    With ``deadline`` (a ``time.time()`` value) digests still running then are abandoned instead
    (:func:`abandon_deferred_md5`); returns False in that case."""
    if deadline is not None:
        wait_all()
        while any(c.engine.md5_pending() for c in Checkpointer._instances.values()):
            if time.time() >= deadline:
                abandon_deferred_md5()
                return False
            time.sleep(0.05)
    for c in list(Checkpointer._instances.values()):
        c.flush()
    return True


_FLUSH_AT_EXIT = [True]


def abandon_deferred_md5():
    """Do not wait for deferred ``.md5`` digests, now or at exit (the time-aware final checkpoint:
    the job's wall-clock limit is near). A digest cut short leaves no ``.md5``; the ``.md5parts``
    written with the archive still verify the resume."""
    _FLUSH_AT_EXIT[0] = False
    errors = []
    for c in list(Checkpointer._instances.values()):
        c.wait()
        e = c.engine.abandon_md5()  # a digest that failed on its own (not by the cancel)
        if e:
            errors.append(e)
    if errors:  # reported, not raised: this runs on the way out of a preempted job
        logger.error("deferred .md5 digest failed before it was abandoned: " + "; ".join(errors))


def _flush_at_exit():
    if not _FLUSH_AT_EXIT[0]:
        return
    try:
        flush_all()
    except Exception as e:  # noqa: BLE001 - interpreter shutdown: report, do not raise
        logger.warning(f"checkpoint flush at exit: {e}")


atexit.register(_flush_at_exit)


def wait_all():
    """Drain every in-flight checkpoint write on this process."""
    out = []
    for c in Checkpointer._instances.values():
        r = c.wait()
        if r is not None:
            out.append(r)
    return out


def fence_all():
    for c in Checkpointer._instances.values():
        c.fence()
    if os.environ.get("PYRECOVER_DEBUG_CKPT") == "1":
        assert_snapshots_landed()


def assert_snapshots_landed():
    """Debug assertion (PYRECOVER_DEBUG_CKPT=1): block until the compute stream has
    passed the snapshot fence and check every staged D2H chunk has completed, i.e. the optimizer
    step that follows cannot mutate parameters that are still being copied out."""
    import torch

    for c in Checkpointer._instances.values():
        if c.staged and c.device_index >= 0:
            torch.cuda.current_stream(c.device_index).synchronize()
            if not c.engine.staged_complete():
                raise RuntimeError("pyrecover: optimizer step would overtake an in-flight checkpoint snapshot")


# ------------------------------------------------------------------------------------------
def _maybe_inject_fault(point: str, path: str):
    """Fault injection for recovery tests: ``PYRECOVER_FAULT=kill_during_write[:<substring>]``
    SIGKILLs this process right after a checkpoint write to a matching path has started (the
    archive is still a ``.tmp`` file), emulating a node failure / hard preemption mid-save."""
    spec = os.environ.get("PYRECOVER_FAULT", "")
    if not spec.startswith("kill_" + point):
        return
    _, _, match = spec.partition(":")
    if match and match not in str(path):
        return
    import signal

    time.sleep(0.01)
    os.kill(os.getpid(), signal.SIGKILL)


_STEP_RE = re.compile(r"ckpt_(\d+)(_final)?")


def ckpt_step(p: Path) -> Tuple[int, int]:
    m = _STEP_RE.search(p.name)
    if not m:
        return (-1, 0)
    return (int(m.group(1)), 1 if m.group(2) else 0)


def is_complete_dir(d: Path) -> bool:
    return (d / ".metadata").exists() and not (d / ".incomplete").exists()


def get_latest_checkpoint(checkpoint_dir: str, distributed: bool = False) -> Optional[str]:
    """Newest checkpoint by mtime, like reference pyrecover/checkpoint.py:371-404; sharded
    directories count only once complete (``.metadata`` written, no ``.incomplete`` marker)."""
    base = Path(checkpoint_dir)
    if not base.exists():
        return None
    if distributed:
        items = [x for x in base.glob("ckpt_*") if x.is_dir() and is_complete_dir(x)]
    else:
        items = [x for x in base.glob("**/*.pt") if x.is_file()]
    if not items:
        return None
    items.sort(key=lambda x: (x.stat().st_mtime, ckpt_step(x)))
    return str(items[-1])


def apply_retention(base: Path, max_keep: int, distributed: bool):
    """Keep the newest ``max_keep`` checkpoints by step number (fixes the reference's
    lexicographic sort); only ``ckpt_*`` entries are ever deleted."""
    if max_keep <= 0:
        return
    if distributed:
        items = [d for d in base.glob("ckpt_*") if d.is_dir() and is_complete_dir(d)]
    else:
        items = [f for f in base.glob("**/*.pt") if f.is_file() and _STEP_RE.search(f.name)]
    items.sort(key=ckpt_step)
    for old in items[:-max_keep]:
        try:
            if old.is_dir():
                shutil.rmtree(old)
            else:
                old.unlink()
                for side in (".md5", ".md5parts"):
                    sp = Path(str(old) + side)
                    if sp.exists():
                        sp.unlink()
        except FileNotFoundError:
            pass
