#!/usr/bin/env python
"""Compare the model weights (and optionally optimizer state) of two checkpoints.

Same CLI and exit codes as reference tests/check_weights_equality.py:59-76, 224-228:

    python tools/check_weights_equality.py ckpt_a ckpt_b [--distributed] [--tolerance 1e-7] [--verbose]
    exit 0: equal   exit 1: differ   exit 2: error

Works for both formats (the reference's ``--distributed`` mode is broken):
vanilla ``.pt`` files and sharded checkpoint directories (ours or ``torch.distributed.checkpoint``
ones) are auto-detected; ``--distributed`` is accepted for CLI parity. Keys are compared after
stripping ``module.``/``_orig_mod.`` prefixes. ``--optimizer`` also compares AdamW moments/steps.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import Dict, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Check if model weights are equal between two checkpoints")
    p.add_argument("checkpoint1", type=str)
    p.add_argument("checkpoint2", type=str)
    p.add_argument("--distributed", action="store_true", help="(auto-detected) sharded checkpoint directories")
    p.add_argument("--tolerance", type=float, default=1e-7)
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--optimizer", action="store_true", help="also compare optimizer state")
    return p.parse_args(argv)


def load_checkpoint(path: str) -> Dict:
    from pyrecover_amd.ckpt.core import strip_prefixes
    from pyrecover_amd.ckpt.sharded import read_sharded_state

    if os.path.isdir(path):
        st = read_sharded_state(path)
        model = st.get("model", {})
        opt = st.get("optimizer") or {}
        return {"model": strip_prefixes(model), "optimizer": opt}
    ck = torch.load(path, map_location="cpu", mmap=True, weights_only=True)
    return {"model": strip_prefixes(ck["model"]), "optimizer": ck.get("optimizer") or {}}


def compare_tensors(a: Dict[str, torch.Tensor], b: Dict[str, torch.Tensor], tol: float,
                    verbose: bool, label: str) -> Tuple[bool, float]:
    ok = True
    ka, kb = set(a), set(b)
    if ka != kb:
        ok = False
        print(f"[{label}] key sets differ: only in 1: {sorted(ka - kb)[:10]}, only in 2: {sorted(kb - ka)[:10]}")
    worst = 0.0
    for k in sorted(ka & kb):
        x, y = a[k], b[k]
        if not isinstance(x, torch.Tensor) or not isinstance(y, torch.Tensor):
            if x != y:
                ok = False
                print(f"[{label}] {k}: values differ ({x!r} vs {y!r})")
            continue
        if x.shape != y.shape:
            ok = False
            print(f"[{label}] {k}: shape {tuple(x.shape)} vs {tuple(y.shape)}")
            continue
        d = (x.float() - y.float()).abs().max().item() if x.numel() else 0.0
        worst = max(worst, d)
        if d > tol:
            ok = False
            print(f"[{label}] {k}: max |diff| = {d:.3e} > {tol:.1e}")
        elif verbose:
            print(f"[{label}] {k}: max |diff| = {d:.3e}")
    return ok, worst


def _flatten_opt(opt: Dict) -> Dict[str, torch.Tensor]:
    out = {}
    for i, st in (opt.get("state") or {}).items():
        for f, v in st.items():
            out[f"state.{int(i)}.{f}"] = torch.as_tensor(v)
    return out


def main(argv=None) -> int:
    args = parse_args(argv)
    try:
        a = load_checkpoint(args.checkpoint1)
        b = load_checkpoint(args.checkpoint2)
    except Exception as e:  # unreadable / missing file
        print(f"error: {e}")
        return 2
    ok, worst = compare_tensors(a["model"], b["model"], args.tolerance, args.verbose, "model")
    if args.optimizer:
        ok2, w2 = compare_tensors(_flatten_opt(a["optimizer"]), _flatten_opt(b["optimizer"]), args.tolerance,
                                  args.verbose, "optimizer")
        ok, worst = ok and ok2, max(worst, w2)
    print(f"{'EQUAL' if ok else 'DIFFERENT'}: {len(a['model'])} tensors, max |diff| = {worst:.3e}")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
