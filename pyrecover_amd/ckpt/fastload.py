"""Native resume path: checkpoint bytes go straight from the file into the live flat buffers.

Replaces the reference's ``torch.load(map_location=device, mmap=True)`` + ``load_state_dict`` +
whole-file MD5 re-read (reference pyrecover/checkpoint.py:137-199) and ``dcp.load``
(:300-368) for models trained with the flat buffers of :mod:`pyrecover_amd.parallel.flat`:

1. *Plan.* The archive's structure is read without touching tensor bytes: ``torch.load(mmap=True,
   weights_only=True)`` for the vanilla ``.pt`` (every storage is a view of one file mapping, so
   its file offset follows from the zip directory) or the manifest of a sharded checkpoint. Each
   parameter / AdamW moment becomes a ``(file offset, nbytes, destination pointer)`` item aimed at
   its slice of ``flat.data`` / ``exp_avg`` / ``exp_avg_sq``.
2. *Read.* :class:`pyrecover_amd._C.CkptReader` reads the file with several threads (O_DIRECT
   when available) into pinned buffers and copies each range H2D into place. Integrity: the
   ``.md5parts`` sidecar (MD5 of every 256 MiB segment) is verified by the same threads from the
   bytes they read; files without it fall back to the reference's whole-file ``.md5`` on a side
   thread.
3. *World > 1.* Rank r reads only the bytes that land in its 1/W of every flat buffer (and hashes
   every W-th segment); the buffers are then completed by one in-place ``all_gather_into_tensor``
   each over RCCL/xGMI, so the file is read once per job instead of once per rank.

Anything the plan cannot place (a dtype/shape mismatch, a tensor outside the flat buffers, a
non-flat model) is copied by torch from the mmap'ed archive, and a checkpoint the planner does not
understand falls back to the generic loader in :mod:`.vanilla` / :mod:`.sharded`.
"""
from __future__ import annotations

import logging
import os
import threading
import time
import zipfile
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .. import _ext
from . import core

logger = logging.getLogger("pyrecover")

# (file offset, nbytes, destination tensor)
Item = Tuple[int, int, torch.Tensor]

ENABLED = os.environ.get("PYRECOVER_FAST_LOAD", "1") == "1"
READ_THREADS = int(os.environ.get("PYRECOVER_CKPT_READ_THREADS", "16"))  # 16 vs 8: md5-verified 7B load 5.5 -> 3.5 s
DIRECT_IO = os.environ.get("PYRECOVER_CKPT_DIRECT", "1") == "1"

_readers: Dict[int, Any] = {}
LAST_STATS: Dict[str, Any] = {}  # stats of the most recent native load (benchmarks, logs)


def _reader(device_index: int):
    if device_index not in _readers:
        _readers[device_index] = _ext.native().CkptReader(device_index)
    return _readers[device_index]


# ------------------------------------------------------------------------------------------
def zip_payloads(path: str) -> Dict[str, Tuple[int, int]]:
    """record name -> (payload file offset, nbytes) of a stored (uncompressed) zip archive."""
    out = {}
    with zipfile.ZipFile(path) as z, open(path, "rb") as f:
        for info in z.infolist():
            if info.compress_type != zipfile.ZIP_STORED:
                raise ValueError(f"{info.filename}: compressed record")
            f.seek(info.header_offset)
            head = f.read(30)
            if head[:4] != b"PK\x03\x04":
                raise ValueError("bad local header")
            nl = int.from_bytes(head[26:28], "little")
            el = int.from_bytes(head[28:30], "little")
            out[info.filename] = (info.header_offset + 30 + nl + el, info.file_size)
    return out


def read_md5parts(path: str) -> Optional[Tuple[int, int, List[str]]]:
    """(segment bytes, file bytes, per-segment md5) from ``<path>.md5parts``, or None."""
    p = Path(str(path) + ".md5parts")
    if not p.exists():
        return None
    lines = p.read_text().split("\n")
    head = lines[0].split()
    if len(head) != 4 or head[0] != "pyrecover-md5parts" or head[1] != "1":
        raise ValueError(f"{p}: unknown md5parts format")
    seg, total = int(head[2]), int(head[3])
    md5s = [x for x in lines[1:] if x]
    if seg != _ext.native().MD5PARTS_SEGMENT_BYTES or len(md5s) != (total + seg - 1) // seg:
        raise ValueError(f"{p}: inconsistent md5parts")
    return seg, total, md5s


def _storage_file_offsets(ckpt, payloads: Dict[str, Tuple[int, int]]) -> Dict[int, int]:
    """storage data_ptr -> file offset for a ``torch.load(mmap=True)`` result: all storages are
    views of ONE mapping of the file, so ptr - file_offset is the same for every storage. The
    i-th storage by address is the i-th data record by offset; the constant is checked for all."""
    ptrs = {}
    for t in core._tensors(ckpt, []):
        st = t.untyped_storage()
        if st.nbytes():
            ptrs[st.data_ptr()] = st.nbytes()
    recs = sorted((off, n) for name, (off, n) in payloads.items() if "/data/" in name and not
                  name.endswith("serialization_id") and n)
    sp = sorted(ptrs.items())
    if len(sp) != len(recs):
        raise ValueError(f"{len(sp)} storages vs {len(recs)} data records")
    base = sp[0][0] - recs[0][0]
    out = {}
    for (ptr, n), (off, rn) in zip(sp, recs):
        if ptr - off != base or n != rn:
            raise ValueError("archive storages are not one contiguous mapping")
        out[ptr] = off
    return out


def _compatible(src: torch.Tensor, dst: torch.Tensor) -> bool:
    return (src.dtype == dst.dtype and src.shape == dst.shape and src.is_contiguous() and dst.is_contiguous()
            and dst.device.type in ("cpu", "cuda"))


def _model_targets(model) -> Dict[str, torch.Tensor]:
    return core.strip_prefixes(core.unwrap(model).state_dict(keep_vars=True))


def _opt_targets(optimizer) -> Optional[List[Dict[str, torch.Tensor]]]:
    """Per saved-parameter-index AdamW moment tensors of a FlatAdamW (else None)."""
    from ..optim.adamw import FlatAdamW

    if not isinstance(optimizer, FlatAdamW):
        return None
    return [optimizer.state[p] for p in optimizer.param_groups[0]["params"]]


def flat_buffers(model, optimizer) -> List[torch.Tensor]:
    m = core.unwrap(model)
    out = []
    flat = getattr(m, "flat", None)
    if flat is not None:
        out.append(flat.data)
    if optimizer is not None and _opt_targets(optimizer) is not None:
        out += [optimizer.exp_avg, optimizer.exp_avg_sq]
        if getattr(optimizer, "master", None) is not None:
            out.append(optimizer.master)
    return out


def _opt_keys(mine: Dict[str, torch.Tensor], saved: Optional[Dict[str, Any]] = None) -> Tuple[str, ...]:
    """Per-parameter optimizer tensors to place: the moments, plus the fp32 master when this run keeps
    one and the checkpoint has it (FlatAdamW master_weights)."""
    keys = ("exp_avg", "exp_avg_sq")
    if "master_param" in mine and (saved is None or "master_param" in saved):
        keys += ("master_param",)
    return keys


# ------------------------------------------------------------------------------------------
class Plan:
    def __init__(self):
        self.files: Dict[str, List[Item]] = {}  # path -> native items
        self.fallback: List[Tuple[torch.Tensor, torch.Tensor]] = []  # (src, dst) copied by torch
        self.model_keys: set = set()  # model keys placed (natively or by fallback)
        self.opt_tensors = False  # AdamW moments placed

    def add(self, path: str, off: int, src: torch.Tensor, dst: torch.Tensor):
        n = dst.numel() * dst.element_size()
        if n:
            self.files.setdefault(path, []).append((off, n, dst))

    def nbytes(self) -> int:
        return sum(n for items in self.files.values() for _, n, _ in items)


def plan_vanilla(path: str, model, optimizer) -> Tuple[Dict[str, Any], Plan]:
    ckpt = torch.load(path, map_location="cpu", mmap=True, weights_only=True)
    offs = _storage_file_offsets(ckpt, zip_payloads(path))
    plan = Plan()

    def place(src, dst):
        st = src.untyped_storage()
        if _compatible(src, dst) and st.data_ptr() in offs:
            plan.add(path, offs[st.data_ptr()] + src.storage_offset() * src.element_size(), src, dst)
        else:
            plan.fallback.append((src, dst))

    tg = _model_targets(model)
    for k, src in core.strip_prefixes(ckpt["model"]).items():
        if k in tg and isinstance(src, torch.Tensor):
            place(src, tg[k].detach())
            plan.model_keys.add(k)
    ot = _opt_targets(optimizer) if "optimizer" in ckpt else None
    if ot is not None:
        osd = ckpt["optimizer"]
        sids = osd["param_groups"][0]["params"]
        if len(sids) == len(ot) and all(sid in osd["state"] for sid in sids):
            for sid, mine in zip(sids, ot):
                for key in _opt_keys(mine, osd["state"][sid]):
                    place(osd["state"][sid][key], mine[key])
            plan.opt_tensors = True
    return ckpt, plan


def _partition(items: Sequence[Item], buffers: Sequence[torch.Tensor], rank: int, world: int) -> Tuple[List, int]:
    """Native read list of this rank: items inside a flat buffer are cut to the rank's 1/W slice
    of that buffer (plus the buffer's < W-byte tail, read by everyone); others are read whole."""
    spans = [(b.data_ptr(), b.numel() * b.element_size()) for b in buffers]
    out = []
    for off, n, dst in items:
        p = dst.data_ptr()
        for base, nb in spans:
            if base <= p and p + n <= base + nb:
                q = nb // world
                rel = p - base
                for lo, hi in ((rank * q, (rank + 1) * q), (world * q, nb)):
                    a, b = max(lo, rel), min(hi, rel + n)
                    if a < b:
                        out.append((off + a - rel, b - a, base + a))
                break
        else:
            out.append((off, n, p))
    return out


def execute(plan: Plan, buffers: Sequence[torch.Tensor], verify: bool = False, md5parts=None,
            whole_md5_path: Optional[str] = None, is_distributed: bool = False) -> Dict[str, Any]:
    """Read every planned item (this rank's share when distributed), verify, complete the flat
    buffers across ranks, then run the torch fallbacks. Raises on any integrity failure."""
    rank, world = (dist.get_rank(), dist.get_world_size()) if is_distributed else (0, 1)
    devs = {d.device for items in plan.files.values() for _, _, d in items}
    if len(devs) > 1:
        raise ValueError(f"destinations on several devices: {devs}")
    dev = devs.pop() if devs else torch.device("cpu")
    dev_index = (dev.index if dev.index is not None else torch.cuda.current_device()) if dev.type == "cuda" else -1
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()  # destination buffers are quiescent
    stats = {"bytes_read": 0, "item_bytes": 0, "read_s": 0.0, "direct": None, "verified": "none"}
    whole = {"ok": True, "err": ""}
    th = None
    if verify and whole_md5_path is not None and md5parts is None and rank == 0:
        from .vanilla import verify_checkpoint

        def _v():
            whole["ok"], whole["err"] = verify_checkpoint(whole_md5_path)
        th = threading.Thread(target=_v, daemon=True)
        th.start()
        stats["verified"] = "md5 (whole file)"
    bad = []
    t0 = time.perf_counter()
    files = dict(plan.files)
    if verify and md5parts is not None and whole_md5_path is not None:
        files.setdefault(whole_md5_path, [])  # segments are hashed even if nothing lands natively
    try:
        for path, items in files.items():
            native = _partition(items, buffers, rank, world)
            stats["item_bytes"] += sum(n for _, n, _ in native)
            hash_segs = []
            if verify and md5parts is not None and path == whole_md5_path:
                hash_segs = [s for s in range(len(md5parts[2])) if s % world == rank]
                stats["verified"] = "md5parts"
            res = _reader(dev_index).read(path, native, hash_segs, READ_THREADS, DIRECT_IO)
            if not res["ok"]:
                raise RuntimeError(f"checkpoint read of {path} failed: {res['error']}")
            stats["bytes_read"] += res["bytes_read"]
            stats["direct"] = res["direct"]
            for s in hash_segs:
                if res["seg_md5"][s] != md5parts[2][s]:
                    bad.append(s)
    finally:
        # resume happens once per job: free the reader's pinned buffers (READ_THREADS x 2 x 64 MiB)
        # instead of holding them for the rest of training
        _readers.pop(dev_index, None)
    stats["read_s"] = time.perf_counter() - t0
    if is_distributed:
        flag = torch.tensor([len(bad)], dtype=torch.int64, device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(flag)
        nbad = int(flag.item())
    else:
        nbad = len(bad)
    if nbad:
        raise RuntimeError(f"Checksum mismatch for checkpoint {whole_md5_path}: {nbad} corrupted segment(s)"
                           + (f" (this rank: {bad[:8]})" if bad else ""))
    if is_distributed and world > 1:
        t1 = time.perf_counter()
        for b in buffers:
            u8 = b.view(-1).view(torch.uint8)
            q = u8.numel() // world
            if q:
                dist.all_gather_into_tensor(u8[:world * q], u8[rank * q:(rank + 1) * q])
        stats["allgather_s"] = time.perf_counter() - t1
    with torch.no_grad():
        for src, dst in plan.fallback:
            dst.copy_(src)
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()
    if th is not None:
        th.join()
    ok = torch.tensor([1 if whole["ok"] else 0], dtype=torch.int64, device=dev if dev.type == "cuda" else "cpu")
    if is_distributed:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok.item()):
        raise RuntimeError(whole["err"] or "Checksum mismatch (reported by rank 0)")
    LAST_STATS.clear()
    LAST_STATS.update(stats)
    return stats


def finish_state(model, optimizer, lr_scheduler, sampler, ckpt, plan: Plan) -> Tuple[int, int]:
    """Everything the native read did not cover: remaining model keys, optimizer hyper-parameters
    and step, scheduler, sampler cursor, RNG streams."""
    m = core.unwrap(model)
    sd = {k: v for k, v in core.strip_prefixes(ckpt["model"]).items() if k not in plan.model_keys}
    with torch.no_grad():
        missing, unexpected = m.load_state_dict(sd, strict=False)  # post hook refreshes W^T shadows
    missing = [k for k in missing if k not in plan.model_keys]
    if missing or unexpected:
        raise RuntimeError(f"checkpoint/model key mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    flat = getattr(m, "flat", None)
    if flat is not None:
        flat.refresh_transposed()
    if optimizer is not None and ckpt.get("optimizer") is not None:
        if plan.opt_tensors:
            optimizer.load_state_dict(ckpt["optimizer"], tensors_loaded=True)
        else:
            optimizer.load_state_dict(ckpt["optimizer"])
    if lr_scheduler is not None and "lr_scheduler" in ckpt:
        sd = dict(ckpt["lr_scheduler"])
        if hasattr(lr_scheduler, "lr_lambdas"):
            sd.setdefault("lr_lambdas", [None] * len(sd.get("base_lrs", lr_scheduler.lr_lambdas)))
        lr_scheduler.load_state_dict(sd)
    if sampler is not None and "sampler_state" in ckpt and hasattr(sampler, "load_state_dict"):
        sampler.load_state_dict(ckpt["sampler_state"])
    core.restore_rng_from(ckpt.get("pyrecover_state"))
    return ckpt.get("epoch", 0), ckpt.get("step", 0)


def load_vanilla(model, optimizer, lr_scheduler, sampler, path: str, verify: bool,
                 is_distributed: bool) -> Tuple[int, int, Dict[str, Any]]:
    ckpt, plan = plan_vanilla(path, model, optimizer)
    md5parts = read_md5parts(path) if verify else None
    if md5parts is not None and md5parts[1] != os.path.getsize(path):
        raise RuntimeError(f"Checksum mismatch for checkpoint {path}: size differs from its md5parts")
    if verify and md5parts is None and not Path(str(path) + ".md5").exists():
        raise RuntimeError(f"[Errno 2] No such file or directory: '{path}.md5'")
    stats = execute(plan, flat_buffers(model, optimizer), verify, md5parts, path, is_distributed)
    epoch, step = finish_state(model, optimizer, lr_scheduler, sampler, ckpt, plan)
    stats["native_bytes"] = plan.nbytes()
    stats["fallback_tensors"] = len(plan.fallback)
    return epoch, step, stats


def plan_sharded(path: str, model, optimizer) -> Tuple[Dict[str, Any], Plan]:
    """Plan of a sharded checkpoint written by this engine (manifest with payload offsets)."""
    import json

    from . import sharded

    p = Path(path)
    mf = p / sharded.MANIFEST
    if not mf.exists():
        raise ValueError("no manifest (not written by pyrecover_amd)")
    manifest = json.loads(mf.read_text())
    native = {k: e for k, e in manifest.items() if "data_offset" in e and
              (k.startswith("model.") or (k.startswith("optimizer.state.") and
                                          k.endswith((".exp_avg", ".exp_avg_sq", ".master_param"))))}
    ckpt = sharded.build_ckpt(sharded.read_sharded_state(path, skip=set(native)))
    plan = Plan()
    tg = _model_targets(model)

    def place(fqn, dst) -> bool:
        e = native.get(fqn)
        if e is None or dst is None:
            return False
        if (str(dst.dtype).replace("torch.", "") != e["dtype"] or list(dst.shape) != list(e["shape"])
                or not dst.is_contiguous()):
            return False
        plan.add(str(p / e["file"]), int(e["data_offset"]), None, dst)
        return True

    placed = set()
    for k in list(ckpt["model"]):
        fqn = "model." + k
        if fqn in native:
            dst = tg.get(core._PREFIX_RE.sub("", k))
            if place(fqn, dst.detach() if dst is not None else None):
                plan.model_keys.add(core._PREFIX_RE.sub("", k))
                placed.add(fqn)
    ot = _opt_targets(optimizer)
    osd = ckpt.get("optimizer")
    if ot is not None and osd is not None and osd.get("param_groups"):
        sids = osd["param_groups"][0]["params"]
        fq = [(f"optimizer.state.{sid}.{key}", mine[key]) for sid, mine in zip(sids, ot)
              for key in _opt_keys(mine)]
        if len(sids) == len(ot) and all(f in native for f, _ in fq):
            for f, dst in fq:
                if place(f, dst):
                    placed.add(f)
            plan.opt_tensors = all(f in placed for f, _ in fq)
    # whatever was skipped but could not be placed is read by the generic path after all
    for fqn in set(native) - placed:
        sharded.fill_value(ckpt, fqn, sharded.read_tensor(p, native[fqn]))
    if not plan.opt_tensors:
        for fqn in placed:
            if fqn.startswith("optimizer."):
                raise ValueError("partial optimizer placement")
    return ckpt, plan
