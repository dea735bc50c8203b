#!/usr/bin/env python
"""Per-kernel register / scratch / occupancy report of a HIP source for gfx950 (hipcc
-Rpass-analysis=kernel-resource-usage), optionally diffed against another version of the file.

  python tools/kernel_resources.py csrc/kernels/attention.hip [--against old.hip] [--filter bf16]
"""
import argparse
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = {"attention.hip": ["-fno-honor-nans", "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]}


def usage(src, inc, flags_of=None):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-I" + inc,
           "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"] + FLAGS.get(os.path.basename(flags_of or src), [])
    r = subprocess.run(cmd, capture_output=True, text=True)
    out, name = {}, None
    for ln in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", ln)
        if m:
            name = m.group(1)
            out[name] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", ln)
        if m and name:
            out[name][m.group(1).split()[0]] = int(m.group(2))
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    return out


def short(n):
    n = re.sub(r"^_ZN3pra\d*\w*?(\d+)", r"\1", n)
    n = re.sub(r"EEEvPK.*", "", n)
    return n.replace("IDF16b", "<bf16,").replace("IDF16_", "<f16,")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--against")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    new = usage(a.src, os.path.join(ROOT, "csrc"))
    old = {}
    if a.against:
        old = {short(k).replace("ILi", "<bf16,Li", 1): v for k, v in usage(a.against, os.path.join(ROOT, "csrc"), a.src).items()}
    fmt = lambda v: f"V{v.get('VGPRs')} A{v.get('AGPRs')} scratch {v.get('ScratchSize')} occ {v.get('Occupancy')} lds {v.get('LDS')}"
    for k, v in new.items():
        s = short(k)
        if a.filter not in s:
            continue
        line = f"{s:48s} {fmt(v)}"
        if a.against:
            o = old.get(s)
            line += "   | before: " + (fmt(o) if o else "-")
        print(line)


if __name__ == "__main__":
    main()
