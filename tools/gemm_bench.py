#!/usr/bin/env python
"""Standalone throughput of the bench's library GEMMs (hipBLASLt via torch.mm) on random bf16
operands, each shape timed back to back (--iters) after warmup, with the committed TunableOp
table (default) or the library heuristic (--no-table). Compares isolated GEMM speed with what the
same shapes reach inside a training step (rocprofv3 kernel stats)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--dim", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=11008)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--qkv-out", type=int, default=0, help="QKV output width (GQA); default 3 x dim")
    ap.add_argument("--hip", action="store_true", help="also time the hand-written NT kernel (gemm_nt_) for "
                                                       "the forward and the shadowed data gradient")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--no-table", action="store_true")
    ap.add_argument("--layouts", action="store_true", help="also time K-contiguous wgrad / transpose variants")
    ap.add_argument("--only", default="", help="comma-separated subset of qkv,wo,w13,w2,head")
    ap.add_argument("--tune", default="", help="tune missing shapes with TunableOp into this table "
                                               "(seeded with the committed table)")
    a = ap.parse_args()
    from pyrecover_amd.utils.gemm_tuning import TABLE, configure_gemm_tuning

    if a.tune:
        import shutil

        if not os.path.exists(a.tune):
            shutil.copy(TABLE, a.tune)
        configure_gemm_tuning("tune", table=a.tune)
        torch.cuda.tunable.read_file(a.tune)
    else:
        configure_gemm_tuning("off" if a.no_table else "auto")
    dev = torch.device("cuda", 0)
    T, Dm, F, V = a.tokens, a.dim, a.ffn, a.vocab
    outs = {"qkv": a.qkv_out or 3 * Dm, "wo": Dm, "w13": 2 * F, "w2": Dm, "head": V}
    ins = {"qkv": Dm, "wo": Dm, "w13": Dm, "w2": F, "head": Dm}
    res = {}
    for name in outs:
        if a.only and name not in a.only.split(","):
            continue
        n_out, n_in = outs[name], ins[name]
        x = torch.randn(T, n_in, device=dev).bfloat16()
        w = torch.randn(n_out, n_in, device=dev).bfloat16()
        dy = torch.randn(T, n_out, device=dev).bfloat16()
        cases = {"fwd": lambda: torch.mm(x, w.t()), "dgrad": lambda: torch.mm(dy, w),
                 "wgrad": lambda: torch.mm(dy.t(), x)}
        if a.layouts:  # K-contiguous (transposed) activations: wgrad as a "TN" GEMM
            dyT, xT, wT = dy.t().contiguous(), x.t().contiguous(), w.t().contiguous()
            cases.update({"wgrad_tn": lambda: torch.mm(dyT, xT.t()), "wgrad_dyT_x": lambda: torch.mm(dyT, x),
                          "dgrad_from_dyT": lambda: torch.mm(dyT.t(), w),
                          "dgrad_wT": lambda: torch.mm(dy, wT.t()),
                          "dgrad_TT": lambda: torch.mm(dyT.t(), wT.t()),
                          "transpose_dy": lambda: dy.t().contiguous(), "transpose_x": lambda: x.t().contiguous()})
        if a.hip and n_out % 256 == 0 and n_in % 256 == 0 and T % 256 == 0:
            from pyrecover_amd import _ext

            C = _ext.native()
            wT = w.t().contiguous()
            y = torch.empty(T, n_out, dtype=x.dtype, device=dev)
            dx = torch.empty(T, n_in, dtype=x.dtype, device=dev)
            cases.update({"fwd_hip": lambda: C.gemm_nt_(x, w, y), "dgrad_hip": lambda: C.gemm_nt_(dy, wT, dx)})
        for cname, fn in cases.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            res[f"{name}_{cname}"] = {"ms": round(ms, 4), "tflops": round(2 * T * n_in * n_out / ms / 1e9, 1)}
        del x, w, dy
    base = [k for k in res if k.split("_", 1)[1] in ("fwd", "dgrad", "wgrad")]
    tot_ms = sum(res[k]["ms"] for k in base if not k.startswith("head")) * 32 + sum(
        res[k]["ms"] for k in base if k.startswith("head"))
    if a.tune:
        torch.cuda.tunable.write_file()
    print(json.dumps({"table": not a.no_table, "gemm_ms_per_step": round(tot_ms, 1), "shapes": res}), flush=True)


if __name__ == "__main__":
    main()
