#!/usr/bin/env python
"""Static instruction mix of HIP kernels, whole kernel and per loop (gfx950 assembly).

Compiles a kernel source to device assembly with the build's flags (pyrecover_amd/_build.py
EXTRA_FLAGS), splits it per kernel symbol, finds the loops (backward branches) and prints, per
kernel and per loop, the count of each opcode class: MFMA, VALU (of which packed fp32 ``v_pk_*``
and ``v_mov_b32``), LDS, global / buffer memory, SALU, waits and barriers. Static counts: a loop body
runs once per iteration, the rest once per block -- which is the distinction a whole-kernel opcode
count (e.g. "330 v_mov_b32 against 32 MFMA") hides.

    python tools/isa_mix.py csrc/kernels/attention.hip --kernels bwd_dkdv_kernelIDF16bLi128ELb1ELi8ELb0 \\
        [--extra-flags "-fno-slp-vectorize"] [--asm /tmp/a.s]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(src, extra, out):
    sys.path.insert(0, ROOT)
    from pyrecover_amd._build import EXTRA_FLAGS, HIPCC, ARCH

    flags = EXTRA_FLAGS.get(os.path.basename(src), []) if extra is None else extra.split()
    cmd = [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", f"-I{ROOT}/csrc", f"-I{ROOT}/csrc/kernels",
           "-DPRA_ATTN_HARNESS=1", "--offload-device-only", "-S", "-o", out, src] + flags
    subprocess.run(cmd, check=True, capture_output=True)


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_mov_b32"):
        return "valu_mov"
    if op.startswith(("v_accvgpr",)):
        return "acc_move"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernels(asm_text):
    for m in re.finditer(r"^(_Z\S+):", asm_text, re.M):
        start = m.end()
        end = asm_text.find(".Lfunc_end", start)
        yield m.group(1), asm_text[start:end].split("\n")


def ops_of(lines):
    out = []
    for ln in lines:
        mm = re.match(r"^\s+([a-z_][a-z0-9_]*)", ln)
        if mm and not ln.strip().startswith((";", ".")):
            out.append(re.sub(r"_(e32|e64|sdwa|dpp)$", "", mm.group(1)))
    return out


def loops(lines):
    labels = {}
    for i, ln in enumerate(lines):
        mm = re.match(r"^(\.LBB\S+):", ln)
        if mm:
            labels[mm.group(1)] = i
    for i, ln in enumerate(lines):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", ln)
        if mm:
            t = mm.group(1) or mm.group(2)
            if labels.get(t, 1 << 30) < i:
                yield labels[t], i


def mix(ops):
    c = collections.Counter(classify(o) for o in ops)
    return {k: c.get(k, 0) for k in ("mfma", "valu", "valu_pk", "valu_mov", "acc_move", "lds", "vmem", "salu",
                                     "wait", "barrier")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--kernels", default="", help="comma list of substrings of kernel symbols")
    ap.add_argument("--extra-flags", default=None, help="override the build's per-file flags")
    ap.add_argument("--asm", default="", help="keep the assembly here")
    a = ap.parse_args()
    out = a.asm or tempfile.mktemp(suffix=".s")
    compile_asm(a.src, a.extra_flags, out)
    text = open(out).read()
    want = [k for k in a.kernels.split(",") if k]
    for name, lines in kernels(text):
        if want and not any(w in name for w in want):
            continue
        print(f"{name[:100]}")
        print(f"  whole kernel: {mix(ops_of(lines))}")
        for lo, hi in loops(lines):
            m = mix(ops_of(lines[lo:hi + 1]))
            if m["mfma"] == 0 and m["lds"] == 0:
                continue  # address / tile-order loops
            per = {k: round(v / m["mfma"], 2) for k, v in m.items() if m["mfma"] and k != "mfma"}
            print(f"  loop lines {lo}-{hi}: {m}  per MFMA: {per}")


if __name__ == "__main__":
    main()
