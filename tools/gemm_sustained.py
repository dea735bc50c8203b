#!/usr/bin/env python
"""Sustained-rate check of hipBLASLt/rocBLAS solutions for one TN GEMM signature from the
TunableOp table: every candidate solution runs in a FRESH process (TunableOp 'use' mode with a
one-entry table), 2 s of back-to-back warm-up on random data, then timed -- the steady-state
clock a training step runs at, unlike TunableOp's short tuning bursts.

  python tools/gemm_sustained.py tn_22016_32768_4096_ld_4096_4096_22016 [--cands a,b,...]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "tuning", "tunableop_gfx950.csv")


def child(sig, sol, secs):
    import time

    import torch

    M, N, K = (int(x) for x in sig.split("_")[1:4])
    lines = [ln for ln in open(TABLE) if ln.startswith("Validator")]
    lines.append(f"GemmTunableOp_BFloat16_TN,{sig},{sol},0.0\n")
    fd, path = tempfile.mkstemp(suffix=".csv")
    os.write(fd, "".join(lines).encode())
    os.close(fd)
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    t.set_filename(path, insert_device_ordinal=False)
    t.read_file(path)
    dev = torch.device("cuda", 0)
    x = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
    w = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    torch.mm(x, w.t())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for _ in range(10):
            torch.mm(x, w.t())
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        torch.mm(x, w.t())
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 30
    os.remove(path)
    print(json.dumps({"sol": sol, "ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sig")
    ap.add_argument("--cands", default="")
    ap.add_argument("--secs", type=float, default=2.0)
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        child(a.sig, a.child, a.secs)
        return
    cands = a.cands.split(",") if a.cands else sorted(
        {ln.split(",")[2] for ln in open(TABLE) if ln.startswith("GemmTunableOp_BFloat16_TN")})
    cur = [ln.split(",")[2] for ln in open(TABLE) if f",{a.sig}," in ln]
    print(f"# {a.sig}: table pick {cur}, {len(cands)} candidates", flush=True)
    for c in cands:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), a.sig, "--child", c, "--secs", str(a.secs)],
                           capture_output=True, text=True, timeout=120)
        out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        print(out[-1] if out else json.dumps({"sol": c, "error": (r.stderr or "")[-300:]}), flush=True)


if __name__ == "__main__":
    main()
