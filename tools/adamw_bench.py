#!/usr/bin/env python
"""Interleaved in-process A/B of the transposing AdamW kernel variants (PRA_ADAMW_T_STRIP, read
per call) over the Llama-2-7B weight matrices (one optimizer step's worth: 32 layers of QKV, O,
W1|W3, W2 plus the output head), random bf16 data; reports ms per step and effective TB/s
(16 B per parameter: p, g, m, v read; p, m, v, p^T written). Results are compared bitwise.

  python tools/adamw_bench.py --values 1,2,4 [--rounds 5] [--layers 32]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--values", default="1,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layers", type=int, default=32)
    a = ap.parse_args()
    from pyrecover_amd import _ext

    C = _ext.native()
    dev = torch.device("cuda", 0)
    g_ = torch.Generator(device=dev).manual_seed(0)
    shapes = [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008)]
    mats = []
    for (r, c) in shapes:  # one set per shape; every layer reuses it (same traffic per call)
        p = (torch.randn(r, c, device=dev, generator=g_) * 0.02).bfloat16()
        grad = (torch.randn(r, c, device=dev, generator=g_) * 1e-3).bfloat16()
        m = (torch.randn(r, c, device=dev, generator=g_) * 1e-4).bfloat16()
        v = (torch.rand(r, c, device=dev, generator=g_) * 1e-6).bfloat16()
        mats.append([p, grad, m, v, torch.empty(c, r, device=dev, dtype=torch.bfloat16)])
    head = [(torch.randn(32000, 4096, device=dev, generator=g_) * 0.02).bfloat16()]
    head += [torch.randn_like(head[0]) * 1e-3, torch.randn_like(head[0]) * 1e-4, torch.rand_like(head[0]) * 1e-6,
             torch.empty(4096, 32000, device=dev, dtype=torch.bfloat16)]
    calls = [mats[i % 4] for i in range(4 * a.layers)] + [head]
    nparam = sum(t[0].numel() for t in calls)

    def step():
        for p, grad, m, v, pt in calls:
            C.adamw_t_(p, grad, m, v, pt, 1e-5, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.7, 1.0, None, None)

    vals = a.values.split(",")
    snaps = {}
    inputs = [t.clone() for t in mats[2]]  # identical inputs for every variant's one-call result
    for x in vals:
        os.environ["PRA_ADAMW_T_STRIP"] = x
        q = [t.clone() for t in inputs]
        C.adamw_t_(q[0], q[1], q[2], q[3], q[4], 1e-5, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.7, 1.0, None, None)
        snaps[x] = q
    for x in vals:  # warm-up
        os.environ["PRA_ADAMW_T_STRIP"] = x
        step()
    torch.cuda.synchronize()
    times = {x: [] for x in vals}
    for _ in range(a.rounds):
        for x in vals:
            os.environ["PRA_ADAMW_T_STRIP"] = x
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            step()
            e1.record()
            torch.cuda.synchronize()
            times[x].append(e0.elapsed_time(e1))
    base = snaps[vals[0]]
    for x in vals:
        med = statistics.median(times[x])
        same = all(torch.equal(s, t) for s, t in zip(snaps[x], base))
        print(f"PRA_ADAMW_T_STRIP={x}: median {med:.2f} ms  min {min(times[x]):.2f} ms  "
              f"{16 * nparam / med / 1e9:.2f} TB/s  ({nparam / 1e9:.2f}B params)  bitwise-equal={same}")


if __name__ == "__main__":
    main()
