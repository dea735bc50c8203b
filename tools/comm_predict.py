#!/usr/bin/env python
"""Predicted exposed gradient communication at N GPUs from a 1-GPU run.

On one GPU the bucket machinery runs without collectives, but the CommTimer still records, per
step, when each bucket's gradients are complete on the compute stream (``ready[b]``) and when the
backward's last kernel ends (``bwd_end``). This tool replays those timestamps against a model of
the in-order collective stream AND of the AdamW updates that wait on each reduced bucket (one
in-order side stream, optim/adamw.py), for each DP mode:

* ``allreduce`` (default DDP): comm FIFO of all-reduces,
      t_ar(b) = latency + bytes_b * 2 (N - 1) / N / busbw,   end_b = max(ready_b, end_{b-1}) + t_ar(b);
  update of bucket b: u_b = max(end_b, u_{b-1}) + t_upd(b), t_upd(b) = adamw_ms * bytes_b / bytes;
* ``shard`` (--shard-optimizer, ZeRO-1): reduce-scatter (half the bus bytes of an all-reduce), an
  update of 1/N of the bucket, and the parameter all-gather, issued on the SAME comm stream behind
  the update; the update of bucket b is released at the next bucket (the attention-window hold),
  so the FIFO is RS_0, RS_1, AG_0, RS_2, AG_1, ..., and an all-gather holds the stream until its
  update is done (head-of-line wait, modelled);
* ``--sparse``: the embedding bucket (the last one) becomes an all-gather of N x B x S (token id,
  row) pairs: t = latency + N n (2 D + 8) (N - 1) / N / busbw + the scatter-add (measured rows).

exposed = max(last comm end, last update end) - bwd_end, minus the same quantity on one GPU (where
the updates already run beside the backward inside the measured step), so
    predicted step (N) = 1-GPU step + exposed(N) - exposed(1).
In the shard mode each rank updates 1/N of every bucket, so the update's cost INSIDE the step
(measured: the 1-GPU step with and without the update kernels, ``update_in_step_ms``) shrinks
with it, assumed in proportion to the bytes:
    predicted step (N, shard) = 1-GPU step - update_in_step (1 - 1/N) + exposed(N) - exposed(1).
A model with transposed weight shadows loses them in the shard mode (models/llama.py); that
difference is not modelled, and the row says so.
``adamw_ms`` is the whole-model update timed alone on this GPU. Not modelled: the CUs RCCL's
kernels take from compute while they overlap it.

  python tools/comm_predict.py --model llama3-8b --batch-per-gpu 1 --world 8 --busbw 150,300,450
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _t(nbytes, factor, busbw_gbps, latency_us):
    return latency_us / 1e3 + nbytes * factor / (busbw_gbps * 1e9) * 1e3  # ms


def simulate(ready, bwd_end, nbytes, world, busbw_gbps, latency_us, adamw_ms=0.0, mode="allreduce",
             sparse_bytes=None, sparse_extra_ms=0.0):
    """(exposed ms, comm ends, update ends) of one step; see the module docstring."""
    total = float(sum(nbytes))
    nb = len(nbytes)
    ar = 2.0 * (world - 1) / world
    half = (world - 1) / world
    upd = [adamw_ms * n / total / (world if mode == "shard" else 1) for n in nbytes]
    comm_t = []
    for b, n in enumerate(nbytes):
        if sparse_bytes is not None and b == nb - 1:
            comm_t.append(_t(sparse_bytes, half, busbw_gbps, latency_us) + sparse_extra_ms)
        elif world <= 1:
            comm_t.append(0.0)
        else:
            comm_t.append(_t(n, ar if mode == "allreduce" else half, busbw_gbps, latency_us))
    sparse_last = sparse_bytes is not None
    if mode == "allreduce" or world <= 1:
        end, u = 0.0, 0.0
        ends, uends = [], []
        for b in range(nb):
            end = max(ready[b], end) + comm_t[b]
            u = max(end, u) + upd[b]
            ends.append(end)
            uends.append(u)
        return max(0.0, max(ends[-1], uends[-1]) - bwd_end), ends, uends
    # shard: RS_b issued at ready_b; AG_b issued after RS_{b+1} (the update is released one bucket
    # later), runs once update b is done; all on one FIFO comm stream. The sparse embedding bucket
    # is reduced whole (no RS / AG), its update sharded like the others.
    order = []
    for b in range(nb):
        order.append(("rs", b))
        if b >= 1:
            order.append(("ag", b - 1))
    order.append(("ag", nb - 1))
    comm_end = 0.0
    rs_end = [0.0] * nb
    u_end = [0.0] * nb
    last_u = 0.0
    ends = []
    for kind, b in order:
        if kind == "rs":
            comm_end = max(ready[b], comm_end) + comm_t[b]
            rs_end[b] = comm_end
            last_u = u_end[b] = max(rs_end[b], last_u) + upd[b]
        else:
            if sparse_last and b == nb - 1:
                comm_end = max(u_end[b], comm_end) + _t(nbytes[b], half, busbw_gbps, latency_us)
            else:
                comm_end = max(u_end[b], comm_end) + comm_t[b]
        ends.append(comm_end)
    return max(0.0, max(comm_end, last_u) - bwd_end), ends, u_end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch-per-gpu", type=int, default=16)
    ap.add_argument("--bucket-mb", type=float, default=256.0)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--busbw", default="150,300,450", help="RCCL all-reduce bus bandwidths, GB/s")
    ap.add_argument("--latency-us", type=float, default=30.0, help="per-collective launch + sync latency")
    ap.add_argument("--json", default="", help="also write the result here")
    ap.add_argument("--modes", default="allreduce,shard", help="DP modes to predict (allreduce, shard)")
    ap.add_argument("--sparse", choices=["auto", "on", "off"], default="auto",
                    help="also predict the sparse embedding exchange (auto: when train.py's auto rule enables it)")
    a = ap.parse_args()

    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.parallel.ddp import GradReducer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = get_preset(a.model, seq_len=a.seq_len)
    torch.manual_seed(0)
    with torch.device(dev):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.bfloat16)
        model = Transformer(cfg)
        torch.set_default_dtype(prev)
    flat = model.flatten_(tokens_per_step=a.batch_per_gpu * a.seq_len)
    reducer = GradReducer(flat, bucket_cap_mb=a.bucket_mb)
    timer = reducer.enable_comm_timing()
    opt = FlatAdamW(flat, lr=1e-5, fused=True)
    opt.enable_overlap(reducer)
    B, S = a.batch_per_gpu, a.seq_len
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    step_ms = []
    for i in range(a.warmup + a.steps):
        timed = i >= a.warmup
        t = torch.randint(0, cfg.vocab_size, (B, S + 1), device=dev, generator=gen)
        if timed:
            timer.begin_step()
        e_end = torch.cuda.Event(enable_timing=True)
        opt.zero_grad()
        loss = model(t[:, :-1], labels=t[:, 1:])
        loss.backward()
        reducer.finish()
        opt.step()
        e_end.record()
        if timed:
            step_ms.append(e_end)
        if not timed:
            timer.steps.clear()
    torch.cuda.synchronize()
    # the same step without the update kernels: what the update costs inside the step
    real_update = opt._update_range
    opt._update_range = lambda *args, **kw: None
    reducer.timer = None  # the recorded steps above stay as they are
    nou = []
    for i in range(a.warmup + a.steps):
        t = torch.randint(0, cfg.vocab_size, (B, S + 1), device=dev, generator=gen)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        opt.zero_grad()
        model(t[:, :-1], labels=t[:, 1:]).backward()
        reducer.finish()
        opt.step()
        e1.record()
        if i >= a.warmup:
            nou.append((e0, e1))
    torch.cuda.synchronize()
    opt._update_range = real_update
    reducer.timer = timer
    noupdate_ms = sum(x.elapsed_time(y) for x, y in nou) / len(nou)
    # the whole-model AdamW update alone on this GPU (the per-bucket updates of the model)
    upd_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rep in range(3):
        upd_ev[0].record()
        opt._update_range(0, flat.numel)
        upd_ev[1].record()
        torch.cuda.synchronize()
    adamw_ms = upd_ev[0].elapsed_time(upd_ev[1])
    # the sparse exchange's local work (sort, row gather, W scatter-adds, copy) on this GPU
    from pyrecover_amd.trainer import _use_sparse_embedding

    n_tok = B * S
    sparse_on = a.sparse == "on" or (a.sparse == "auto" and _use_sparse_embedding("auto", a.world, n_tok,
                                                                                   cfg.vocab_size))
    sparse_bytes = a.world * n_tok * (2 * cfg.dim + 8) if sparse_on else None
    sparse_extra = 0.0
    if sparse_on:
        emb = torch.zeros(cfg.vocab_size + 1, cfg.dim, device=dev)
        rows = torch.randn(n_tok, cfg.dim, device=dev).bfloat16()
        ids = torch.randint(0, cfg.vocab_size, (n_tok,), device=dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for rep in range(3):  # the first pass loads the kernels
            ev[0].record()
            torch.sort(ids)
            sel = emb.index_select(0, ids)
            for _ in range(a.world):
                emb.index_add_(0, ids, rows.float())
            emb.index_copy_(0, ids, sel)
            ev[1].record()
            torch.cuda.synchronize()
        sparse_extra = ev[0].elapsed_time(ev[1])
    nb = timer.nb
    ready = [0.0] * nb
    bwd_end = 0.0
    span = 0.0
    for c, e_end in zip(timer.steps, step_ms):
        t0 = c["t0"]
        for b in range(nb):
            ready[b] += t0.elapsed_time(c["ready"][b]) / len(timer.steps)
        bwd_end += t0.elapsed_time(c["bwd_end"]) / len(timer.steps)
        span += t0.elapsed_time(e_end) / len(timer.steps)
    nbytes = timer.bytes
    exp1, _, _ = simulate(ready, bwd_end, nbytes, 1, 1.0, 0.0, adamw_ms)
    rows = []
    variants = [(m, False) for m in a.modes.split(",")] + ([(m, True) for m in a.modes.split(",")] if sparse_on else [])
    for mode, sp in variants:
        for bw in [float(x) for x in a.busbw.split(",")]:
            exp, ends, uends = simulate(ready, bwd_end, nbytes, a.world, bw, a.latency_us, adamw_ms, mode,
                                        sparse_bytes if sp else None, sparse_extra if sp else 0.0)
            pred = span + exp - exp1
            if mode == "shard":
                pred -= max(0.0, span - noupdate_ms) * (1.0 - 1.0 / a.world)
            shadows = bool(getattr(flat, "shadow_sites", ())) and mode == "shard"
            rows.append({"mode": mode + ("+sparse" if sp else "") + (" (shadows lost: not modelled)" if shadows else ""),
                         "busbw_gbps": bw,
                         "comm_end_ms": round(max(ends), 2), "update_end_ms": round(max(uends), 2),
                         "exposed_ms": round(exp, 2), "predicted_step_ms": round(pred, 1),
                         "predicted_scaling_eff": round(span / pred, 4)})
    out = {"model": a.model, "batch_per_gpu": B, "seq_len": S, "world": a.world, "bucket_mb": a.bucket_mb,
           "buckets": nb, "grad_gib": round(sum(nbytes) / 2**30, 3), "step_ms_1gpu": round(span, 1),
           "bwd_end_ms": round(bwd_end, 1), "first_ready_ms": round(ready[0], 1), "last_ready_ms": round(ready[-1], 1),
           "adamw_alone_ms": round(adamw_ms, 2), "exposed_1gpu_ms": round(exp1, 2),
           "step_ms_1gpu_without_update": round(noupdate_ms, 1), "update_in_step_ms": round(span - noupdate_ms, 1),
           "sparse_exchange_mib": round(sparse_bytes / 2**20, 1) if sparse_bytes else None,
           "sparse_local_ms": round(sparse_extra, 2), "latency_us": a.latency_us, "rows": rows,
           "ready_ms": [round(x, 2) for x in ready], "bucket_mib": [round(x / 2**20, 1) for x in nbytes]}
    print(f"{a.model} B{B} S{S}: 1-GPU step {span:.1f} ms, backward ends at {bwd_end:.1f} ms; {nb} buckets "
          f"({out['grad_gib']} GiB), ready {ready[0]:.1f} .. {ready[-1]:.1f} ms; AdamW alone {adamw_ms:.1f} ms "
          f"(1-GPU update tail {exp1:.2f} ms; the step without the update {noupdate_ms:.1f} ms)")
    print(f"| mode | busbw GB/s | comm ends ms | updates end ms | exposed ms | predicted step ms (N={a.world}) | "
          f"scaling eff |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['mode']} | {r['busbw_gbps']:.0f} | {r['comm_end_ms']} | {r['update_end_ms']} | {r['exposed_ms']} | "
              f"{r['predicted_step_ms']} | {r['predicted_scaling_eff']} |")
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
