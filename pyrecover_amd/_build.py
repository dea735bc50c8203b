"""In-tree native build for pyrecover_amd._C (gfx950 only).

Compiles every HIP kernel in ``csrc/kernels`` with ``hipcc --offload-arch=gfx950`` (pure HIP,
no torch headers), the torch/pybind adapter ``csrc/bindings.cpp`` and the host runtime in
``csrc/runtime`` (checkpoint engine), and links them into ``pyrecover_amd/_C*.so`` next to this
file, so the shared object travels with the repository snapshot. No hipify, no CUDA paths.

Usage: ``python -m pyrecover_amd._build [-j N] [--force]``.
Objects are cached in ``build/`` and rebuilt when a source or any header is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PYRECOVER_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(ROOT, "pyrecover_amd", "_C" + suffix)


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max([os.path.getmtime(h) for h in hs] + [0.0])


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r


# Per-file code-generation flags. attention.hip: no NaN semantics for fmaxf (drops the canonicalising
# v_max before every max on MFMA results) and no SLP packing of f32 adds (packed f32 VALU beside
# MFMAs costs more issue cycles than the scalar form).
# -amdgpu-mfma-vgpr-form: the one-wave-per-SIMD backward kernel keeps its loop-carried dK/dV sums in
# VGPRs; with AGPR-form MFMAs the compiler copies them between the two files around every step.
EXTRA_FLAGS = {"attention.hip": ["-fno-honor-nans", "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
               "attention_bwd_fused.hip": ["-fno-honor-nans", "-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build(jobs: int = 8, force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, libdir, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-mcode-object-version=5",
              "-D__HIP_PLATFORM_AMD__=1", f"-I{CSRC}"]
    torch_flags = [f"-I{p}" for p in inc] + [f"-I{py_inc}", "-DTORCH_EXTENSION_NAME=_C",
                                             "-DTORCH_API_INCLUDE_EXTENSION_H", "-DUSE_ROCM=1",
                                             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-unused-result"]
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hosts = [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + sorted(
        glob.glob(os.path.join(CSRC, "dist", "*.cpp")))
    hdr_t = _newest_header()
    tasks = []
    objs = []
    for src in kernels + hosts:
        obj = os.path.join(BUILD, os.path.relpath(src, CSRC).replace(os.sep, "_") + ".o")
        objs.append(obj)
        stale = force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t)
        if not stale:
            continue
        if src.endswith(".hip"):
            cmd = [HIPCC] + common + EXTRA_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
        else:  # host translation units (torch + pybind headers); compiled as HIP host code
            cmd = [HIPCC] + common + torch_flags + ["-x", "hip", "-c", src, "-o", obj]
        tasks.append(cmd)
    if tasks:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for r in ex.map(_run, tasks):
                if verbose and (r.stdout or r.stderr):
                    print(r.stdout + r.stderr)
    out = ext_path()
    if tasks or force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs + [
            f"-L{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-Wl,-rpath,{libdir}", "-lz", "-lcrypto", "-lpthread", f"-L{os.path.join(ROCM, 'lib')}", "-lroctx64"]
        _run(link)
        os.replace(out + ".tmp", out)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.jobs, a.force, a.verbose))


if __name__ == "__main__":
    sys.exit(main())
