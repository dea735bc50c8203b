"""Forward / data-gradient GEMMs (NT: both operands K-contiguous) of the 7B step: the hand-written
MFMA kernel (csrc/kernels/gemm_nt.hip, C.gemm_nt_) against hipBLASLt (torch.mm with the step's
tuned solution table), and the fused epilogues against library GEMM + our separate kernel:

  plain     C.gemm_nt_(x, w, y)                          vs torch.mm(x, w.t())
  swiglu    C.gemm_nt_(x, w13, gu, 1, a)                 vs torch.mm + C.swiglu_fwd
  swiglu_b  C.gemm_nt_(dy, w2t, gu, 2)                   vs torch.mm + C.swiglu_bwd (in place)
  rope      C.gemm_nt_(x, wqkv, qkv, 3, tab=..)          vs torch.mm + C.rope_

Numerics first (fp32 oracle; fused vs unfused-on-the-same-kernel bitwise), then timing: arms
interleaved in one process, median of rounds. One JSON line per case.

    python tools/gemm_nt_bench.py [--tokens 32768] [--rounds 5] [--cases plain,swiglu,...]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402

# (name, N = out features, K = in features): y[T, N] = x[T, K] w[N, K]^T
PLAIN = [("qkv_fwd", 12288, 4096), ("o_fwd", 4096, 4096), ("w13_fwd", 22016, 4096), ("w2_fwd", 4096, 11008),
         ("qkv_dgrad", 4096, 12288), ("o_dgrad", 4096, 4096), ("w13_dgrad", 4096, 22016), ("w2_dgrad", 11008, 4096),
         ("head_fwd", 32000, 4096), ("head_dgrad", 4096, 32000)]


def timeit(fn, iters, s, e):
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default="plain,swiglu,swiglu_b,rope")
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning("auto")
    C = _ext.native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    T = args.tokens
    cases = set(args.cases.split(","))
    sel = set(args.shapes.split(",")) if args.shapes else None
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def rnd(*shape):
        return (torch.rand(*shape, device=dev) * 2 - 1).bfloat16()

    def run_arms(name, flop, arms, extra=None):
        for f in arms.values():  # warm
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in arms}
        for _ in range(args.rounds):
            for k, f in arms.items():
                res[k].append(timeit(f, args.iters, s, e))
        out = {"case": name, "tokens": T}
        for k, v in res.items():
            med = statistics.median(v)
            out[k + "_us"] = round(med, 1)
            out[k + "_tflops"] = round(flop / med / 1e6, 1)
        if extra:
            out.update(extra)
        print(json.dumps(out), flush=True)

    if "plain" in cases:
        for name, N, K in PLAIN:
            if sel and name not in sel:
                continue
            x, w = rnd(T, K), rnd(N, K) * 0.05
            y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            C.gemm_nt_(x, w, y)
            ref = torch.mm(x.float(), w.float().t())
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-2, (name, err)
            del ref
            y2 = torch.empty_like(y)

            arms = {"lib": lambda: torch.mm(x, w.t(), out=y2), "hip": lambda: C.gemm_nt_(x, w, y)}
            run_arms(name, 2.0 * T * N * K, arms, {"rel_err": round(err, 5)})
            del x, w, y, y2
            torch.cuda.empty_cache()
    F, D = 11008, 4096
    if "swiglu" in cases:
        x, w13 = rnd(T, D), rnd(2 * F, D) * 0.05
        gu = torch.empty(T, 2 * F, device=dev, dtype=torch.bfloat16)
        a = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
        C.gemm_nt_(x, w13, gu, 1, a)
        gu0 = torch.empty_like(gu)
        C.gemm_nt_(x, w13, gu0)
        a0 = C.swiglu_fwd(gu0)
        bit = bool(torch.equal(gu, gu0) and torch.equal(a, a0))
        gul = torch.empty_like(gu)

        def lib():
            torch.mm(x, w13.t(), out=gul)
            C.swiglu_fwd(gul)
        run_arms("swiglu_fwd", 2.0 * T * 2 * F * D, {"lib+kernel": lib, "hip_unfused": lambda: (C.gemm_nt_(x, w13, gu0), C.swiglu_fwd(gu0)),
                                                    "hip_fused": lambda: C.gemm_nt_(x, w13, gu, 1, a)},
                 {"bitwise_vs_unfused": bit})
        del x, w13, gu, a, gu0, a0, gul
        torch.cuda.empty_cache()
    if "swiglu_b" in cases:
        dy, w2t = rnd(T, D), rnd(F, D) * 0.05
        gu = rnd(T, 2 * F)
        g1 = gu.clone()
        C.gemm_nt_(dy, w2t, g1, 2)
        da = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
        C.gemm_nt_(dy, w2t, da)
        g2 = gu.clone()
        C.swiglu_bwd(da, g2, g2)
        bit = bool(torch.equal(g1, g2))
        work = gu.clone()
        dal = torch.empty_like(da)

        def lib():
            torch.mm(dy, w2t.t(), out=dal)
            C.swiglu_bwd(dal, work, work)
        run_arms("swiglu_bwd", 2.0 * T * F * D, {"lib+kernel": lib, "hip_unfused": lambda: (C.gemm_nt_(dy, w2t, da), C.swiglu_bwd(da, work, work)),
                                                "hip_fused": lambda: C.gemm_nt_(dy, w2t, work, 2)},
                 {"bitwise_vs_unfused": bit})
        del dy, w2t, gu, g1, g2, da, work, dal
        torch.cuda.empty_cache()
    if "rope" in cases:
        S, Dh, nq, nk = 2048, 128, 4096, 1024
        N = nq + 2 * nk
        x, w = rnd(T, D), rnd(N, D) * 0.05
        pos = torch.arange(S, device=dev, dtype=torch.float32)
        inv = 1.0 / (10000.0 ** (torch.arange(0, Dh, 2, device=dev, dtype=torch.float32) / Dh))
        ang = torch.outer(pos, inv)
        tab = torch.stack([ang.cos(), ang.sin()], -1).contiguous()
        q1 = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
        C.gemm_nt_(x, w, q1, 3, None, tab, S, Dh, nq + nk)
        q2 = torch.empty_like(q1)
        C.gemm_nt_(x, w, q2)
        C.rope_(q2, nq + nk, tab, Dh, S, 0, False)
        bit = bool(torch.equal(q1, q2))
        ql = torch.empty_like(q1)

        def lib():
            torch.mm(x, w.t(), out=ql)
            C.rope_(ql, nq + nk, tab, Dh, S, 0, False)
        run_arms("qkv_rope", 2.0 * T * N * D, {"lib+kernel": lib, "hip_unfused": lambda: (C.gemm_nt_(x, w, q2), C.rope_(q2, nq + nk, tab, Dh, S, 0, False)),
                                              "hip_fused": lambda: C.gemm_nt_(x, w, q1, 3, None, tab, S, Dh, nq + nk)},
                 {"bitwise_vs_unfused": bit})


if __name__ == "__main__":
    main()
