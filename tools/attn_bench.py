#!/usr/bin/env python
"""Attention kernel microbenchmark: forward / backward TFLOP/s of the HIP flash kernels on the
bench shape (default B=4, S=2048, Hq=Hkv=32, D=128, causal), on random data (rule: never on zeros).

FLOP convention (causal halves): fwd 4*B*H*S^2*D/2, bwd (dkdv + dq kernels, recompute included)
14*B*H*S^2*D/2 -- the work the kernels actually do -- and the "model" bwd convention 10*... .
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=32)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--noncausal", action="store_true")
    a = ap.parse_args()
    from pyrecover_amd import _ext

    C = _ext.native()
    dev = torch.device("cuda", 0)
    B, S, Hq, Hkv, D = a.B, a.S, a.Hq, a.Hkv, a.D
    causal = not a.noncausal
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev).bfloat16()
    nq, nk = Hq * D, Hkv * D
    q = qkv[:, :nq].view(B, S, Hq, D)
    k = qkv[:, nq:nq + nk].view(B, S, Hkv, D)
    v = qkv[:, nq + nk:].view(B, S, Hkv, D)
    do = torch.randn(B, S, Hq, D, device=dev).bfloat16()
    dqkv = torch.empty_like(qkv)
    dq = dqkv[:, :nq].view(B, S, Hq, D)
    dk = dqkv[:, nq:nq + nk].view(B, S, Hkv, D)
    dv = dqkv[:, nq + nk:].view(B, S, Hkv, D)
    scale = 1 / math.sqrt(D)

    def fwd():
        return C.attn_fwd(q, k, v, scale, causal)

    o, lse = fwd()

    def bwd():
        C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    tf = timeit(fwd)
    tb = timeit(bwd)
    frac = 0.5 if causal else 1.0
    base = B * Hq * S * S * D * frac
    out = {"shape": dict(B=B, S=S, Hq=Hq, Hkv=Hkv, D=D, causal=causal), "fwd_ms": round(tf, 4),
           "bwd_ms": round(tb, 4), "fwd_tflops": round(4 * base / tf / 1e9, 1),
           "bwd_tflops_model": round(10 * base / tb / 1e9, 1), "bwd_tflops_executed": round(14 * base / tb / 1e9, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
