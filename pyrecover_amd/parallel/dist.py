"""Process-group runtime: SLURM / torchrun / single-process detection, device binding.

Function names mirror reference dist_utils.py (``maybe_init_distributed``, ``get_rank``,
``is_rank0``, ``is_distributed_activated``, ``log_rank0``, ``maybe_cleanup_distributed``,
``get_slurm_job_end_time_env``; reference dist_utils.py:14-101) but the runtime also accepts
torchrun-style env (RANK/WORLD_SIZE/LOCAL_RANK), picks RCCL (torch backend "nccl" on ROCm) on GPU
and gloo on CPU, and never calls ``exit()`` on a bad environment (it raises).

One process per GPU; the collective layer for gradients is RCCL over xGMI.
"""
from __future__ import annotations

import datetime
import logging
import os
from typing import Optional, Tuple

import torch

logger = logging.getLogger("pyrecover")

_STATE = {"rank": 0, "world": 1, "local_rank": 0, "initialized": False, "backend": None, "reducer": None}


def set_reducer_settings(bucket_mb=None, allreduce=None, shard_optimizer=None, sparse_embedding=None):
    """Record how this run splits and reduces gradients (bucket size in MiB, all-reduce backend,
    sharded optimizer, sparse embedding exchange): bucket boundaries decide how RCCL splits each
    message and so the order in which an element's W contributions are summed. Recorded in every
    checkpoint (``pyrecover_state.reduction``) and compared on resume. Replaces what an earlier
    call recorded (one training run per call)."""
    cur = {}
    for k, v in (("bucket_mb", bucket_mb), ("allreduce", allreduce), ("shard_optimizer", shard_optimizer),
                 ("sparse_embedding", sparse_embedding)):
        if v is not None:
            cur[k] = v
    _STATE["reducer"] = cur


def is_distributed_slurm_env() -> bool:
    return "SLURM_PROCID" in os.environ and int(os.environ.get("SLURM_NTASKS", "1")) > 1


def is_torchrun_env() -> bool:
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) >= 1


def is_distributed_activated() -> bool:
    return "DISTRIBUTED_RUN" in os.environ


def _env_rank_world_local() -> Optional[Tuple[int, int, int]]:
    if is_torchrun_env() and int(os.environ["WORLD_SIZE"]) > 1:
        return int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ.get("LOCAL_RANK", 0))
    if is_distributed_slurm_env():
        return (int(os.environ["SLURM_PROCID"]), int(os.environ["SLURM_NTASKS"]),
                int(os.environ.get("SLURM_LOCALID", 0)))
    return None


def get_rank() -> int:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank()
    return 0


def get_world_size() -> int:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_world_size()
    return 1


def is_rank_eq(rank: int) -> bool:
    return get_rank() == rank


def is_rank0() -> bool:
    return get_rank() == 0


def local_rank() -> int:
    return _STATE["local_rank"]


def gpu_index(lrank: int) -> int:
    """Visible GPU of a local rank (one process per GPU).

    * ``PYRECOVER_LOCAL_DEVICE=<i>`` pins every rank to GPU i (rehearsing the multi-rank path on
      one GPU; use with PYRECOVER_DIST_BACKEND=gloo).
    * One visible device (SLURM per-task isolation: ``--gpus-per-task=1`` / ``--gpu-bind``, or
      ROCR/HIP_VISIBLE_DEVICES set per rank): device 0, whatever SLURM_LOCALID says.
    * Otherwise every node GPU is visible, as in reference dist_utils.py:47,55: GPU ``lrank``. More
      local ranks than visible GPUs is refused here (the reference's ``set_device`` fails loudly
      too), instead of letting two ranks share a GPU and RCCL fail later with an unrelated error.

    ``torch.cuda.device_count()`` does not initialise the GPU on this image."""
    o = os.environ.get("PYRECOVER_LOCAL_DEVICE")
    if o not in (None, ""):
        return int(o)
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    if n <= 0:
        return lrank
    if n == 1:
        return 0
    if lrank >= n:
        raise RuntimeError(
            f"local rank {lrank} (SLURM_LOCALID={os.environ.get('SLURM_LOCALID')}, "
            f"LOCAL_RANK={os.environ.get('LOCAL_RANK')}) has no GPU of its own: only {n} are visible. "
            f"Launch at most {n} tasks per node, bind one GPU per task, or set PYRECOVER_LOCAL_DEVICE "
            f"to share one deliberately")
    return lrank


def rccl_pg_options():
    """Process-group options for RCCL: collectives on a high-priority HIP stream, so a bucket's
    all-reduce workgroups are dispatched ahead of queued backward GEMM tiles and start together on
    every rank instead of spinning behind compute. ``PYRECOVER_RCCL_HIGH_PRIORITY=0`` turns it off."""
    if os.environ.get("PYRECOVER_RCCL_HIGH_PRIORITY", "1") != "1" or not hasattr(torch.distributed,
                                                                                  "ProcessGroupNCCL"):
        return None
    opts = torch.distributed.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


# Reduction-order settings of RCCL: the algorithm, protocol and channel count decide how a bucket
# is split and in which order each element's W contributions are added, so two runs (or a run and
# its resumption after a requeue) reduce identically only when these match. RCCL's tuner picks them
# per message size and topology unless they are set.
RCCL_ORDER_KEYS = ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "NCCL_NCHANNELS_PER_NET_PEER",
                   "RCCL_MSCCL_ENABLE", "RCCL_MSCCLPP_ENABLE", "NCCL_IB_DISABLE", "NCCL_P2P_DISABLE")
# What PYRECOVER_RCCL_DETERMINISTIC=1 pins (only keys the user left unset): ring all-reduce with the
# Simple protocol over a fixed channel count, no MSCCL/MSCCL++ algorithm substitution. The ring
# visits ranks in a fixed order, so every element is summed in the same order on every step.
RCCL_PINNED = {"NCCL_ALGO": "Ring", "NCCL_PROTO": "Simple", "NCCL_MIN_NCHANNELS": "16", "NCCL_MAX_NCHANNELS": "16",
               "RCCL_MSCCL_ENABLE": "0", "RCCL_MSCCLPP_ENABLE": "0"}


def pin_rccl_order(environ=None) -> dict:
    """With PYRECOVER_RCCL_DETERMINISTIC=1, set RCCL_PINNED's keys the environment leaves unset (before
    the process group exists). Returns what was set."""
    env = os.environ if environ is None else environ
    if env.get("PYRECOVER_RCCL_DETERMINISTIC", "0") != "1":
        return {}
    done = {}
    for k, v in RCCL_PINNED.items():
        if k not in env:
            env[k] = v
            done[k] = v
    return done


def rccl_order_settings(environ=None) -> dict:
    """The reduction-order settings in effect (recorded in every checkpoint's pyrecover_state)."""
    env = os.environ if environ is None else environ
    out = {k: env[k] for k in RCCL_ORDER_KEYS if k in env}
    out["world_size"] = get_world_size() if _STATE.get("initialized") else 1
    out["backend"] = _STATE.get("backend") or "none"
    out["rccl_order_pinned"] = env.get("PYRECOVER_RCCL_DETERMINISTIC", "0") == "1"
    for k, v in (_STATE.get("reducer") or {}).items():
        out[k] = v
    return out


_NEWER_KEYS = ("rccl_order_pinned", "bucket_mb", "allreduce", "shard_optimizer", "sparse_embedding")


def compare_rccl_order(saved: Optional[dict], current: Optional[dict] = None) -> list:
    """Differences between a checkpoint's recorded reduction settings and this run's (empty when
    they match or nothing was recorded). A difference means the resumed run is not guaranteed to
    reduce gradients in the same order as the run that wrote the checkpoint."""
    if not saved:
        return []
    cur = rccl_order_settings() if current is None else current
    # keys a checkpoint of an older version does not carry are not differences
    keys = sorted(k for k in set(saved) | set(cur) if k in saved or k not in _NEWER_KEYS)
    return [f"{k}: saved {saved.get(k, '<unset>')!r}, now {cur.get(k, '<unset>')!r}" for k in keys
            if saved.get(k) != cur.get(k)]


def maybe_init_distributed(activate_distributed: bool, backend: Optional[str] = None,
                           timeout_s: float = 1800.0) -> Tuple[int, int]:
    """Returns (local_rank, world_size). Initializes the process group when a multi-process
    environment is present (SLURM with >1 tasks, or torchrun with WORLD_SIZE>1), or when
    ``--distributed`` is given under torchrun with one process (a 1-rank group)."""
    env = _env_rank_world_local()
    if activate_distributed:
        os.environ["DISTRIBUTED_RUN"] = "1"
        if env is None and is_torchrun_env():  # torchrun with one process: a 1-rank group, as asked
            env = (int(os.environ["RANK"]), 1, int(os.environ.get("LOCAL_RANK", 0)))
    if env is None:
        if activate_distributed:
            raise RuntimeError("--distributed was given but no multi-process SLURM/torchrun environment was found")
        if torch.cuda.is_available():
            torch.cuda.set_device(0)
        return 0, 1
    rank, world, lrank = env
    os.environ["DISTRIBUTED_RUN"] = "1"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    use_gpu = torch.cuda.is_available()
    if backend is None:
        backend = os.environ.get("PYRECOVER_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")  # nccl = RCCL
    dev_index = gpu_index(lrank)
    if use_gpu:
        torch.cuda.set_device(dev_index)
    if not torch.distributed.is_initialized():
        kw = {}
        if backend == "nccl":
            pinned = pin_rccl_order()
            if pinned:
                log_rank0(f"PYRECOVER_RCCL_DETERMINISTIC=1: pinned {pinned}")
            kw["device_id"] = torch.device("cuda", dev_index)
            opts = rccl_pg_options()
            if opts is not None:
                kw["pg_options"] = opts
        torch.distributed.init_process_group(backend=backend, rank=rank, world_size=world,
                                             timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _STATE.update(rank=rank, world=world, local_rank=lrank, initialized=True, backend=backend)
    # every rank, like reference dist_utils.py:56-59 (plus the bound device)
    print(f"[Rank {rank}] world_size={world}, local_rank={lrank}, "
          f"device={'cuda:%d' % dev_index if use_gpu else 'cpu'}, pid={os.getpid()}", flush=True)
    log_rank0(f"Distributed initialized: backend={backend} world_size={world} rank={rank} local_rank={lrank}")
    return lrank, world


def maybe_cleanup_distributed():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def barrier():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()


def log_rank(msg, rank):
    if is_rank_eq(rank):
        logger.info(msg)


def log_rank0(msg):
    log_rank(msg, 0)


def get_slurm_job_end_time_env() -> Optional[float]:
    """SLURM_JOB_END_TIME (UNIX seconds) or None (reference dist_utils.py:93-101)."""
    val = os.environ.get("SLURM_JOB_END_TIME")
    if val is not None:
        try:
            return float(val)
        except ValueError:
            pass
    return None
