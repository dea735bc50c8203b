#!/usr/bin/env python
"""fp32 attention: the HIP kernels (csrc/kernels/attention_f32.hip) against the torch math path they
replaced (ops.reference.attention_ref + autograd), forward and forward+backward, one process.

    python tools/attn_f32_bench.py [--B 4 --S 2048 --Hq 32 --Hkv 32 --D 128]
"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=32)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from pyrecover_amd import _ext
    from pyrecover_amd.ops import reference as R

    C = _ext.native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, S, Hq, Hkv, D = a.B, a.S, a.Hq, a.Hkv, a.D
    q = torch.randn(B, S, Hq, D, device=dev)
    k = torch.randn(B, S, Hkv, D, device=dev)
    v = torch.randn(B, S, Hkv, D, device=dev)
    do = torch.randn(B, S, Hq, D, device=dev)
    scale = 1 / math.sqrt(D)

    def hip_fwd():
        return C.attn_fwd(q, k, v, scale, True)

    def hip_fb():
        o, lse = C.attn_fwd(q, k, v, scale, True)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True)

    def torch_fwd():
        with torch.no_grad():
            return R.attention_ref(q, k, v, True, scale)

    def torch_fb():
        qq, kk, vv = (t.detach().requires_grad_() for t in (q, k, v))
        o = R.attention_ref(qq, kk, vv, True, scale)
        torch.autograd.grad(o, (qq, kk, vv), do)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / a.iters)
        return statistics.median(ts)

    fwd_flops = 4 * B * Hq * S * S * D / 2  # causal
    res = {"shape": dict(B=B, S=S, Hq=Hq, Hkv=Hkv, D=D, causal=True, dtype="fp32")}
    for name, fn, fl in (("hip_fwd", hip_fwd, fwd_flops), ("hip_fwd_bwd", hip_fb, 3.5 * fwd_flops),
                         ("torch_fwd", torch_fwd, fwd_flops), ("torch_fwd_bwd", torch_fb, 3.5 * fwd_flops)):
        ms = timeit(fn)
        res[name] = {"ms": round(ms, 3), "TF_model": round(fl / ms / 1e9, 1)}
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
