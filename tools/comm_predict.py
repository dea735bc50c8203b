#!/usr/bin/env python
"""Predicted exposed gradient communication at N GPUs from a 1-GPU run.

On one GPU the bucket machinery runs without collectives, but the CommTimer still records, per
step, when each bucket's gradients are complete on the compute stream (``ready[b]``) and when the
backward's last kernel ends (``bwd_end``). This tool replays those timestamps against a model of
RCCL's in-order collective stream:

    t_b   = latency + bytes_b * 2 (N - 1) / N / busbw          (ring all-reduce, bus bandwidth)
    end_b = max(ready_b, end_{b-1}) + t_b
    exposed = max(0, end_last - bwd_end)

for a list of bus bandwidths, so a later N-GPU run (bench.py prints ``comm.exposed_comm_ms`` and the
per-bucket bus bandwidth it measured) can be checked against a stated prediction. Not modelled: the
CUs RCCL's kernels take from compute while they overlap it, and the per-bucket AdamW updates that
wait on reduced buckets (they run beside the backward on a side stream).

  python tools/comm_predict.py --model llama2-7b --batch-per-gpu 16 --world 8 --busbw 150,300,450
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def simulate(ready, bwd_end, nbytes, world, busbw_gbps, latency_us):
    end = 0.0
    ends = []
    for r, nb in zip(ready, nbytes):
        t = latency_us / 1e3 + nb * 2.0 * (world - 1) / world / (busbw_gbps * 1e9) * 1e3  # ms
        end = max(r, end) + t
        ends.append(end)
    return max(0.0, ends[-1] - bwd_end), ends


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
    rows = []
    for bw in [float(x) for x in a.busbw.split(",")]:
        exp, ends = simulate(ready, bwd_end, nbytes, a.world, bw, a.latency_us)
        busy = sum(a.latency_us / 1e3 + n * 2.0 * (a.world - 1) / a.world / (bw * 1e9) * 1e3 for n in nbytes)
        rows.append({"busbw_gbps": bw, "allreduce_busy_ms": round(busy, 2), "exposed_comm_ms": round(exp, 2),
                     "predicted_step_ms": round(span + exp, 1),
                     "predicted_scaling_eff": round(span / (span + exp), 4)})
    out = {"model": a.model, "batch_per_gpu": B, "seq_len": S, "world": a.world, "bucket_mb": a.bucket_mb,
           "buckets": nb, "grad_gib": round(sum(nbytes) / 2**30, 3), "step_ms_1gpu": round(span, 1),
           "bwd_end_ms": round(bwd_end, 1), "first_ready_ms": round(ready[0], 1), "last_ready_ms": round(ready[-1], 1),
           "latency_us": a.latency_us, "rows": rows,
           "ready_ms": [round(x, 2) for x in ready], "bucket_mib": [round(x / 2**20, 1) for x in nbytes]}
    print(f"{a.model} B{B} S{S}: 1-GPU step {span:.1f} ms, backward ends at {bwd_end:.1f} ms; {nb} buckets "
          f"({out['grad_gib']} GiB), ready {ready[0]:.1f} .. {ready[-1]:.1f} ms")
    print(f"| busbw GB/s | all-reduce busy ms | exposed ms | predicted step ms (N={a.world}) | scaling eff |")
    print("|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['busbw_gbps']:.0f} | {r['allreduce_busy_ms']} | {r['exposed_comm_ms']} | {r['predicted_step_ms']} | "
              f"{r['predicted_scaling_eff']} |")
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
