"""Gradient-bucket size autotune.

``--bucket-cap-mb auto`` (train.py) / ``--bucket-mb auto`` (bench.py): before the first step, every
rank all-reduces a few probe sizes on the real process group, the per-size time is the MAX over
ranks, and a latency / bandwidth model

    t(s) = alpha + s / beta

is fitted by least squares. The cap is the smallest power-of-two MiB whose fixed cost alpha is at
most ``overhead`` (10%) of its transfer time, s >= alpha * beta * (1 - overhead) / overhead: larger
buckets only delay the first collective of the backward, smaller ones pay the per-collective
latency again and again. On xGMI the ring all-reduce is per-link bound (7 links per GPU), so beta is
measured, not assumed. Every rank takes rank 0's choice (a broadcast), so the bucket layout -- and
with it the reduction order -- is the same on all ranks.

The reference relies on DDP's fixed 25 MiB default (reference train.py:107-115); a probe on the job's
own group replaces that guess.
"""
import time
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

PROBE_MB = (4, 16, 64, 256)


def fit_latency_bandwidth(samples: Sequence[Tuple[float, float]]) -> Tuple[float, float]:
    """Least-squares fit of t = alpha + bytes / beta over (bytes, seconds) samples -> (alpha s, beta B/s).
    A non-positive slope (all sizes equally fast) gives beta = inf; a negative intercept clamps to 0."""
    n = len(samples)
    if n < 2:
        raise ValueError("need at least two probe sizes")
    mx = sum(b for b, _ in samples) / n
    my = sum(t for _, t in samples) / n
    sxx = sum((b - mx) ** 2 for b, _ in samples)
    sxy = sum((b - mx) * (t - my) for b, t in samples)
    slope = sxy / sxx if sxx > 0 else 0.0
    alpha = max(0.0, my - slope * mx)
    beta = 1.0 / slope if slope > 0 else float("inf")
    return alpha, beta


def choose_bucket_mb(alpha: float, beta: float, overhead: float = 0.1, lo_mb: int = 16, hi_mb: int = 512) -> int:
    """Smallest power-of-two MiB in [lo_mb, hi_mb] with alpha <= overhead * t(s)."""
    if beta == float("inf") or alpha <= 0.0:
        return lo_mb
    need = alpha * beta * (1.0 - overhead) / overhead / 2 ** 20
    mb = lo_mb
    while mb < need and mb < hi_mb:
        mb *= 2
    return mb


def probe_allreduce(device: torch.device, dtype: torch.dtype = torch.bfloat16, sizes_mb: Sequence[int] = PROBE_MB,
                    iters: int = 3, group=None) -> List[Tuple[float, float]]:
    """(bytes, seconds) per probe size: the mean of `iters` timed all-reduces after one warmup, MAX over
    ranks. Collective: every rank of `group` must call it with the same arguments."""
    esz = torch.empty((), dtype=dtype).element_size()
    buf = torch.zeros(max(sizes_mb) * 2 ** 20 // esz, dtype=dtype, device=device)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    out = []
    for mb in sizes_mb:
        x = buf[: mb * 2 ** 20 // esz]
        dist.all_reduce(x, group=group)
        sync()
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=group)
        sync()
        dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64,
                          device=device if device.type == "cuda" else "cpu")
        dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
        out.append((float(x.numel() * esz), float(dt.item())))
    del buf
    return out


class _ProbeFlat:
    """The part of FlatParams the xGMI engine touches: a gradient buffer it may re-point."""

    def __init__(self, n: int, dtype: torch.dtype, device: torch.device):
        self.grad = torch.zeros(n, dtype=dtype, device=device)

    def rebind_grad(self, new: torch.Tensor):
        self.grad = new


def probe_xgmi(device: torch.device, dtype: torch.dtype = torch.bfloat16, sizes_mb: Sequence[int] = PROBE_MB,
               iters: int = 3, group=None) -> List[Tuple[float, float]]:
    """probe_allreduce through the direct xGMI engine (parallel/xgmi.py): one single-bucket engine per
    probe size over a scratch buffer, timed launch -> wait -> end_step, MAX over ranks. Collective."""
    from .xgmi import XgmiAllReduce

    esz = torch.empty((), dtype=dtype).element_size()
    out = []
    for mb in sizes_mb:
        n = mb * 2 ** 20 // esz
        eng = XgmiAllReduce(_ProbeFlat(n, dtype, device), [(0, n)], group)

        def once():
            eng.launch(0).wait()
            eng.end_step()

        once()
        torch.cuda.synchronize(device)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            once()
        torch.cuda.synchronize(device)
        dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=device)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
        out.append((float(n * esz), float(dt.item())))
        del eng
    return out


def _summary(samples, world) -> dict:
    alpha, beta = fit_latency_bandwidth(samples)
    return {"alpha_us": round(alpha * 1e6, 1),
            "algbw_gbps": None if beta == float("inf") else round(beta / 1e9, 2),
            "busbw_gbps": None if beta == float("inf") else round(beta / 1e9 * 2 * (world - 1) / world, 2),
            "probe": [{"mb": round(b / 2 ** 20), "ms": round(t * 1e3, 3)} for b, t in samples]}


def autotune_bucket_mb(device: torch.device, dtype: torch.dtype = torch.bfloat16, group=None,
                       sizes_mb: Sequence[int] = PROBE_MB, iters: int = 3, overhead: float = 0.1,
                       backend: str = "rccl", flat=None) -> Tuple[int, dict]:
    """Probe, fit and choose; returns (bucket MiB, report). Single process: the 256 MiB default.

    RCCL is always probed. On a GPU group the xGMI engine is probed too (``backend="xgmi"``: the
    bucket size is chosen from ITS fit; otherwise it is reported next to RCCL's, and a probe that
    cannot run -- e.g. per-task GPU isolation -- is reported as such), so the first multi-GPU run logs
    both bus bandwidths."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) < 2:
        return 256, {"world": 1, "chosen_mb": 256}
    world = dist.get_world_size(group)
    samples = probe_allreduce(device, dtype, sizes_mb, iters, group)
    report = {"world": world, "rccl": _summary(samples, world)}
    chosen_from = samples
    if device.type == "cuda":
        try:
            xs = probe_xgmi(device, dtype, sizes_mb, iters, group)
            report["xgmi"] = _summary(xs, world)
            if backend == "xgmi":
                chosen_from = xs
        except Exception as e:  # noqa: BLE001 - decided collectively inside XgmiAllReduce (raises on all ranks)
            if backend == "xgmi":
                raise
            report["xgmi"] = f"not available: {str(e).splitlines()[0][:160]}"
    alpha, beta = fit_latency_bandwidth(chosen_from)
    mb = choose_bucket_mb(alpha, beta, overhead)
    choice = torch.tensor([mb], dtype=torch.int64, device=device if device.type == "cuda" else "cpu")
    dist.broadcast(choice, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    mb = int(choice.item())
    report.update({"chosen_mb": mb, "chosen_for": backend if device.type == "cuda" else "rccl",
                   "alpha_us": report["rccl"]["alpha_us"], "busbw_gbps": report["rccl"]["busbw_gbps"],
                   "probe": report["rccl"]["probe"]})
    return mb, report


def parse_bucket_arg(v):
    """argparse type for --bucket-cap-mb / --bucket-mb: a size in MiB or 'auto'."""
    if isinstance(v, str) and v.strip().lower() == "auto":
        return "auto"
    f = float(v)
    if f <= 0:
        raise ValueError("bucket size must be positive")
    return f
