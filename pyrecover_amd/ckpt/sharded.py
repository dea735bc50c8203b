"""Sharded checkpoints (``--use-torch-distributed-ckpt``): one directory per checkpoint, every
rank writes a disjoint, byte-balanced share of the (replicated) state.

Replaces reference pyrecover/checkpoint.py:218-368 (which delegates to
``torch.distributed.checkpoint``) with a native writer that produces the SAME on-disk layout, so
the reference's ``dcp.load`` path can still read our checkpoints:

* ``__{rank}_0.distcp``: concatenated ``torch.save`` blobs, one per tensor leaf, plus
  ``torch.save``'d python values (rank 0), written by the C++ engine from the pinned snapshot;
* ``.metadata``: a pickled ``torch.distributed.checkpoint.metadata.Metadata`` (FQNs
  ``model.<param>``, ``optimizer.state.<i>.{step,exp_avg,exp_avg_sq}``,
  ``optimizer.param_groups.0.<k>``, ``lr_scheduler.<k>``, ``metadata.{epoch,step}``, ...);
* ``pyrecover_manifest.json``: where each tensor's raw bytes sit (file, offset, dtype, shape), used
  by the fast loader (parallel reads straight into the target tensors, no unpickling).

Model keys carry no ``module.`` prefix, so save/load works across world sizes.
A checkpoint directory is only considered by ``latest`` once rank 0 has written ``.metadata``
after every rank finished its shard (``.incomplete`` marker until then).
"""
from __future__ import annotations

import io
import json
import logging
import os
import pickle
import struct
import time
import uuid
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import core
from .serialization import plan_archive, torch_save_bytes

logger = logging.getLogger("pyrecover")

MANIFEST = "pyrecover_manifest.json"


def flatten_state(obj, prefix: str = "", out: Optional[Dict[str, Any]] = None, keypath=()):
    """dcp-style flattening: nested dicts/lists -> {"a.b.0.c": leaf} and the key-path map."""
    if out is None:
        out = {}
    if isinstance(obj, dict) and obj:
        for k, v in obj.items():
            flatten_state(v, f"{prefix}.{k}" if prefix else str(k), out, keypath + (str(k) if not isinstance(k, int)
                                                                                        else str(k),))
    elif isinstance(obj, list) and obj and not all(isinstance(x, (int, float, str, bool)) for x in obj):
        for i, v in enumerate(obj):
            flatten_state(v, f"{prefix}.{i}", out, keypath + (i,))
    else:
        out[prefix] = (obj, keypath)
    return out


def _rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def assign_owners(items: Dict[str, Tuple[Any, tuple]], world: int) -> Dict[str, int]:
    """Deterministic byte-balanced assignment of tensor leaves to ranks (largest first);
    python values go to rank 0 (like dcp's coordinator)."""
    owners = {}
    load = [0] * world
    tens = [(k, v[0]) for k, v in items.items() if isinstance(v[0], torch.Tensor)]
    tens.sort(key=lambda kv: (-kv[1].numel() * kv[1].element_size(), kv[0]))
    for k, t in tens:
        r = min(range(world), key=lambda i: (load[i], i))
        owners[k] = r
        load[r] += t.numel() * t.element_size()
    for k, v in items.items():
        if not isinstance(v[0], torch.Tensor):
            owners[k] = 0
    return owners


def _local_header_data_offset(blob_head: bytes) -> int:
    """Offset of the payload inside a zip local file header."""
    sig, = struct.unpack_from("<I", blob_head, 0)
    if sig != 0x04034B50:
        raise ValueError("not a zip local header")
    nl, el = struct.unpack_from("<HH", blob_head, 26)
    return 30 + nl + el


def save_ckpt_distributed(model, optimizer, lr_scheduler=None, sampler=None, step: int = 0, epoch: Optional[int] = None,
                          checkpoint_path: str = "ckpt", max_keep: int = 3, verify: bool = True,
                          is_distributed: bool = False, rank: int = 0, *, async_save: bool = False,
                          fsync: bool = True, extra_state=None) -> str:
    rank, world = _rank_world()
    path = Path(checkpoint_path)
    if is_distributed:
        dist.barrier()
    core.wait_all()
    finalize_pending()
    core.prepare_optimizer_state(optimizer)  # collective: a sharded optimizer gathers its moments
    rngs = core.gather_rng_states() if is_distributed else None  # collective: every rank's streams
    state = core.build_state(model, optimizer, lr_scheduler, sampler, step, epoch, extra_state, rngs)
    # dcp key layout: "metadata" holds epoch/step (reference checkpoint.py:254-258)
    dstate: Dict[str, Any] = {"model": state["model"], "optimizer": state["optimizer"],
                              "metadata": {"epoch": epoch, "step": step}}
    if "lr_scheduler" in state:
        dstate["lr_scheduler"] = state["lr_scheduler"]
    if "sampler_state" in state:
        dstate["sampler"] = state["sampler_state"]
    dstate["pyrecover_state"] = {"rng": state["pyrecover_state"]["rng"],
                                 "format": state["pyrecover_state"]["format"],
                                 "reduction": state["pyrecover_state"]["reduction"]}
    if rngs is not None:
        dstate["pyrecover_state"]["rng_per_rank"] = {str(r): st for r, st in enumerate(rngs)}
    items = flatten_state(dstate)
    owners = assign_owners(items, world)
    mine = {k: v for k, v in items.items() if owners[k] == rank}
    if rank == 0:
        path.mkdir(parents=True, exist_ok=True)
        (path / ".incomplete").write_text(str(time.time()))
    if is_distributed:
        dist.barrier()
    dev = next(core.unwrap(model).parameters()).device
    ck = core.Checkpointer.get(dev)
    staged = ck.stage({k: v[0] for k, v in mine.items()})
    wr_items, keep, order = [], [], []
    pos = {k: i for i, k in enumerate(items)}
    for k in sorted(mine, key=pos.__getitem__):
        val = staged[k]
        if isinstance(val, torch.Tensor):
            recs, kp = plan_archive(val, "archive")
            wr_items.append(("zip", recs))
            keep.append(kp)
        else:
            b = torch_save_bytes(val)
            import ctypes

            buf = ctypes.create_string_buffer(b, len(b))
            keep.append(buf)
            wr_items.append(("raw", ctypes.addressof(buf), len(b)))
        order.append(k)
    fname = f"__{rank}_0.distcp"
    meta_local = []
    for k in order:
        v = items[k][0]
        if isinstance(v, torch.Tensor):
            meta_local.append((k, "tensor", str(v.dtype).replace("torch.", ""), list(v.shape)))
        else:
            meta_local.append((k, "bytes", None, None))
    pend = {"path": str(path), "rank": rank, "world": world, "fname": fname, "meta": meta_local, "items": items,
            "max_keep": max_keep, "distributed": is_distributed, "t0": time.perf_counter()}
    # the Job caches its result, so whoever drains the engine first (poll_all / wait_all / a later
    # save) cannot take this shard's layout away from finalize_pending
    pend["job"] = ck.write(str(path / fname), wr_items, False, fsync, (staged, keep), None)
    _PENDING.append(pend)
    if not async_save:
        finalize_pending()
    elif is_distributed:
        dist.barrier()
    return str(path)


_PENDING: List[Dict[str, Any]] = []


def finalize_pending():
    """Collective on all ranks: wait for this process's shard, gather shard layouts to rank 0,
    write ``.metadata`` + manifest, drop ``.incomplete``, apply retention."""
    while _PENDING:
        pend = _PENDING.pop(0)
        res = pend["job"].wait()
        if len(res["items"]) != len(pend["meta"]):
            raise RuntimeError(f"shard {pend['fname']} of {pend['path']}: {len(res['items'])} records written, "
                               f"{len(pend['meta'])} expected")
        # payload offset of each tensor blob's "data/0" record (the fast loader reads only those bytes)
        data0 = {}
        for name, doff, _ in res["records"]:
            if name.endswith("/data/0"):
                for i, (off, ln) in enumerate(res["items"]):
                    if off <= doff < off + ln:
                        data0[i] = doff
        local = [(k, kind, dt, shape, pend["fname"], off, ln, data0.get(i))
                 for i, ((k, kind, dt, shape), (off, ln)) in enumerate(zip(pend["meta"], res["items"]))]
        gathered = [local]
        if pend["distributed"]:
            gathered = [None] * pend["world"]
            dist.all_gather_object(gathered, local)
        if pend["rank"] == 0:
            _write_metadata(Path(pend["path"]), pend["items"], [e for g in gathered for e in g])
            core.apply_retention(Path(pend["path"]).parent, pend["max_keep"], distributed=True)
            logger.info(f"sharded checkpoint {pend['path']} complete in {time.perf_counter() - pend['t0']:.2f}s")
        if pend["distributed"]:
            dist.barrier()


def _write_metadata(path: Path, items, entries):
    from torch.distributed.checkpoint.filesystem import _StorageInfo
    from torch.distributed.checkpoint.metadata import (BytesStorageMetadata, ChunkStorageMetadata, Metadata,
                                                       MetadataIndex, StorageMeta, TensorProperties,
                                                       TensorStorageMetadata)

    sd_meta, storage, planner, manifest = {}, {}, {}, {}
    for (k, kind, dt, shape, fname, off, ln, data_off) in entries:
        val, keypath = items[k]
        planner[k] = keypath
        if kind == "tensor":
            t = val
            size = torch.Size(shape)
            sd_meta[k] = TensorStorageMetadata(properties=TensorProperties(dtype=t.dtype), size=size,
                                               chunks=[ChunkStorageMetadata(offsets=torch.Size([0] * len(size)),
                                                                            sizes=size)])
            storage[MetadataIndex(fqn=k, offset=torch.Size([0] * len(size)), index=0)] = _StorageInfo(fname, off, ln)
            manifest[k] = {"file": fname, "offset": off, "length": ln, "dtype": dt, "shape": shape}
            if data_off is not None:
                manifest[k]["data_offset"] = data_off
        else:
            sd_meta[k] = BytesStorageMetadata()
            storage[MetadataIndex(fqn=k)] = _StorageInfo(fname, off, ln)
    md = Metadata(state_dict_metadata=sd_meta, planner_data=planner, storage_data=storage,
                  storage_meta=StorageMeta(checkpoint_id=str(path), save_id=str(uuid.uuid4())), version="1.0.0")
    tmp = path / ".metadata.tmp"
    with open(tmp, "wb") as f:
        pickle.dump(md, f)
        f.flush()
        os.fsync(f.fileno())
    (path / (MANIFEST + ".tmp")).write_text(json.dumps(manifest))
    os.replace(path / (MANIFEST + ".tmp"), path / MANIFEST)
    os.replace(tmp, path / ".metadata")
    inc = path / ".incomplete"
    if inc.exists():
        inc.unlink()


# ------------------------------------------------------------------------------------------
def _read_blob(path: Path, fname: str, off: int, ln: int) -> bytes:
    with open(path / fname, "rb") as f:
        f.seek(off)
        return f.read(ln)


def _load_value(path: Path, sinfo) -> Any:
    return torch.load(io.BytesIO(_read_blob(path, sinfo.relative_path, sinfo.offset, sinfo.length)),
                      map_location="cpu", weights_only=True)


def _tensor_from_manifest(path: Path, ent) -> torch.Tensor:
    """Fast path for our own shards: read only the payload bytes of the blob."""
    with open(path / ent["file"], "rb") as f:
        f.seek(ent["offset"])
        head = f.read(4096)
        # the first record of a torch.save blob is data.pkl; walk records until "data/0"
        pos = 0
        while True:
            sig, = struct.unpack_from("<I", head, pos) if pos + 4 <= len(head) else (0,)
            if sig != 0x04034B50:
                raise ValueError("unexpected blob layout")
            csize, = struct.unpack_from("<I", head, pos + 18)
            nl, el = struct.unpack_from("<HH", head, pos + 26)
            name = head[pos + 30:pos + 30 + nl].decode()
            data_off = pos + 30 + nl + el
            if name.endswith("/data/0"):
                dtype = getattr(torch, ent["dtype"])
                n = 1
                for s in ent["shape"]:
                    n *= s
                nbytes = n * torch.empty((), dtype=dtype).element_size()
                f.seek(ent["offset"] + data_off)
                buf = bytearray(f.read(nbytes))
                return torch.frombuffer(buf, dtype=dtype).view(ent["shape"]) if nbytes else \
                    torch.empty(ent["shape"], dtype=dtype)
            if csize == 0xFFFFFFFF:
                raise ValueError("zip64 record before data/0")
            pos = data_off + csize
            if pos + 30 > len(head):
                f.seek(ent["offset"] + pos)
                head = head[:pos] + f.read(4096)


class _MetadataUnpickler(pickle.Unpickler):
    """Unpickles a dcp ``.metadata`` file while refusing every global that is not part of the dcp
    metadata schema (dataclasses of torch.distributed.checkpoint, torch.Size, dtypes, containers),
    so a crafted checkpoint directory cannot execute code on load."""

    _MODULES = ("torch.distributed.checkpoint.metadata", "torch.distributed.checkpoint.filesystem",
                "torch.distributed.checkpoint.planner")
    _GLOBALS = {("torch", "Size"), ("collections", "OrderedDict"), ("builtins", "set"), ("builtins", "frozenset"),
                ("builtins", "slice"), ("copyreg", "_reconstructor"), ("builtins", "object"), ("enum", "Enum"),
                ("torch._utils", "_rebuild_tensor_v2"), ("torch.storage", "_load_from_bytes"),
                ("torch", "device"), ("torch", "memory_format"), ("torch", "layout"),
                ("torch.serialization", "_get_layout"), ("pathlib", "PosixPath"), ("pathlib", "PurePosixPath")}

    def find_class(self, module, name):
        if module in self._MODULES or (module, name) in self._GLOBALS:
            return super().find_class(module, name)
        if module == "torch" and isinstance(getattr(torch, name, None), (torch.dtype, torch.layout,
                                                                         torch.memory_format)):
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"checkpoint metadata references {module}.{name}, which is not allowed")


def read_metadata(path) -> Any:
    with open(Path(path) / ".metadata", "rb") as f:
        return _MetadataUnpickler(f).load()


def read_tensor(p: Path, ent) -> torch.Tensor:
    return _tensor_from_manifest(p, ent)


def read_sharded_state(path: str, skip=()) -> Dict[str, Any]:
    """Rebuild the nested state dict (CPU tensors) of a sharded checkpoint (ours or dcp's).
    Entries named in ``skip`` are not read (None placeholders; the fast loader places them)."""
    p = Path(path)
    md = read_metadata(p)  # a dcp Metadata object (written by us or by torch.distributed.checkpoint)
    manifest = {}
    if (p / MANIFEST).exists():
        manifest = json.loads((p / MANIFEST).read_text())
    flat: Dict[str, Any] = {}
    for idx, sinfo in md.storage_data.items():
        k = idx.fqn
        if k in skip:
            flat[k] = None
        elif k in manifest:
            flat[k] = _tensor_from_manifest(p, manifest[k])
        else:
            flat[k] = _load_value(p, sinfo)
    # unflatten with planner_data key paths (ints index lists, strings index dicts)
    out: Dict[str, Any] = {}
    for k, v in flat.items():
        keypath = md.planner_data.get(k, tuple(k.split(".")))
        cur = out
        for i, part in enumerate(keypath):
            last = i == len(keypath) - 1
            nxt_container = None if last else ([] if isinstance(keypath[i + 1], int) else {})
            if isinstance(cur, list):
                while len(cur) <= part:
                    cur.append(None)
                if last:
                    cur[part] = v
                else:
                    if cur[part] is None:
                        cur[part] = nxt_container
                    cur = cur[part]
            else:
                if last:
                    cur[part] = v
                else:
                    if part not in cur:
                        cur[part] = nxt_container
                    cur = cur[part]
    return _fix_lists(out)


def _fix_lists(o):
    if isinstance(o, dict):
        return {k: _fix_lists(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_fix_lists(v) for v in o]
    return o


def build_ckpt(st: Dict[str, Any]) -> Dict[str, Any]:
    """dcp-layout state -> the vanilla checkpoint dict layout (reference checkpoint.py:254-258)."""
    model_sd = st.get("model", {})
    opt_sd = st.get("optimizer")
    if opt_sd is not None:
        # optimizer.state keys come back as strings ("0", "1", ...): torch wants ints
        opt_sd = {"state": {int(k): v for k, v in opt_sd.get("state", {}).items()},
                  "param_groups": opt_sd.get("param_groups", [])}
    ckpt = {"model": model_sd, "optimizer": opt_sd, "epoch": st.get("metadata", {}).get("epoch", 0),
            "step": st.get("metadata", {}).get("step", 0)}
    if "lr_scheduler" in st:
        ckpt["lr_scheduler"] = st["lr_scheduler"]
    if "sampler" in st:
        ckpt["sampler_state"] = st["sampler"]
    if "pyrecover_state" in st:
        ckpt["pyrecover_state"] = st["pyrecover_state"]
    return ckpt


def fill_value(ckpt: Dict[str, Any], fqn: str, value):
    """Put a dcp FQN's value into a :func:`build_ckpt` dict."""
    parts = fqn.split(".")
    if parts[0] == "model":
        ckpt["model"][".".join(parts[1:])] = value
    elif parts[:2] == ["optimizer", "state"]:
        ckpt["optimizer"]["state"][int(parts[2])][".".join(parts[3:])] = value
    else:
        raise KeyError(fqn)


def load_ckpt_distributed(model, optimizer, lr_scheduler=None, sampler=None, checkpoint_path: str = "latest",
                          experiment_dir: str = ".", verify: bool = True, is_distributed: bool = False,
                          rank: int = 0) -> Tuple[int, int]:
    if is_distributed:
        dist.barrier()
    core.wait_all()
    finalize_pending()
    if checkpoint_path == "latest":
        checkpoint_path = core.get_latest_checkpoint(str(experiment_dir), distributed=True)
        if checkpoint_path is None:
            raise RuntimeError(f"No checkpoint found in {experiment_dir}")
    from . import fastload

    stats = None
    try:
        plan = fastload.plan_sharded(checkpoint_path, model, optimizer) if fastload.ENABLED else None
    except (ValueError, KeyError, OSError) as e:  # not our layout: generic path
        logger.info(f"sharded fast load not applicable ({e}); using the generic reader")
        plan = None
    if plan is not None:
        ckpt, pl = plan
        stats = fastload.execute(pl, fastload.flat_buffers(model, optimizer), False, None, None, is_distributed)
        epoch, step = fastload.finish_state(model, optimizer, lr_scheduler, sampler, ckpt, pl)
    else:
        from .vanilla import load_state_into

        ckpt = build_ckpt(read_sharded_state(checkpoint_path))
        epoch, step = load_state_into(model, optimizer, lr_scheduler, sampler, ckpt)
    if stats is not None:
        logger.info(f"native read: {stats['bytes_read'] / 2**30:.2f} GiB in {stats['read_s']:.2f}s"
                    + (f", all-gather {stats['allgather_s']:.2f}s" if "allgather_s" in stats else ""))
    if is_distributed:
        dist.barrier()
    logger.info(f"Distributed checkpoint loaded from {checkpoint_path} (epoch {epoch}, step {step})")
    return epoch, step
