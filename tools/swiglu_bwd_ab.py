"""Interleaved in-process A/B of the swiglu_bwd_t kernel generations (csrc/kernels/elementwise.hip,
PRA_SWIGLU_BWD = 0: one row in flight per lane, 1: hoisted loads, 2: hoisted loads over two
64x64 tiles) at the 7B batch-16 shape (T = 32768 tokens, F = 11008). Every generation must be
bit-identical to generation 0. Prints one JSON line per (variant, round) and a summary line.

    python tools/swiglu_bwd_ab.py [--tokens 32768] [--ffn 11008] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--ffn", type=int, default=11008)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    C = _ext.native()
    dev = torch.device("cuda", 0)
    T, F = args.tokens, args.ffn
    torch.manual_seed(0)
    gu0 = torch.randn(T, 2 * F, device=dev).bfloat16()
    dy = torch.randn(T, F, device=dev).bfloat16()
    gu = torch.empty_like(gu0)
    variants = ["0", "1", "2"]
    ref = None
    for v in variants:  # correctness: bitwise equal outputs
        os.environ["PRA_SWIGLU_BWD"] = v
        gu.copy_(gu0)
        guT = C.swiglu_bwd_t_(dy, gu)
        torch.cuda.synchronize()
        if ref is None:
            ref = (gu.clone(), guT.clone())
        else:
            assert torch.equal(gu, ref[0]) and torch.equal(guT, ref[1]), f"variant {v} differs"
        assert torch.equal(guT, gu.t())
    nbytes = T * F * 2 + 2 * T * 2 * F * 2 + T * 2 * F * 2  # dy + gu read, gu + guT written
    res = {v: [] for v in variants}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.rounds):
        for v in variants:
            os.environ["PRA_SWIGLU_BWD"] = v
            for _ in range(3):
                C.swiglu_bwd_t_(dy, gu)
            s.record()
            for _ in range(args.iters):
                C.swiglu_bwd_t_(dy, gu)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / args.iters
            res[v].append(us)
            print(json.dumps({"variant": v, "round": r, "us": round(us, 1),
                              "TBps": round(nbytes / 1e9 / us * 1e3, 2)}), flush=True)
    print(json.dumps({"summary": {v: {"median_us": round(statistics.median(x), 1), "min_us": round(min(x), 1),
                                      "TBps_median": round(nbytes / 1e9 / statistics.median(x) * 1e3, 2)}
                                  for v, x in res.items()}, "tokens": T, "ffn": F}), flush=True)


if __name__ == "__main__":
    main()
