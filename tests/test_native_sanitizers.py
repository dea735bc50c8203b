"""Host-side sanitizer runs of the native checkpoint engine (ASan/UBSan debug build,
race detection on the writer / MD5 threads). The engine core is header-only host C++
(csrc/runtime/ckpt_engine.h); tests/native/ckpt_engine_selftest.cpp drives it in CPU mode
(no GPU calls) through staging, two back-to-back archive writes reusing the pinned pool, and the
error path. GPU sanitizers are not available on this pool, so only host code is instrumented."""
import os
import shutil
import subprocess
import zipfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
SRC = os.path.join(ROOT, "tests", "native", "ckpt_engine_selftest.cpp")


def _build(tmp_path, flags, name):
    cxx = shutil.which("g++")
    if cxx is None or not os.path.exists(os.path.join(ROCM, "include", "hip", "hip_runtime_api.h")):
        pytest.skip("g++ / ROCm headers not available")
    exe = str(tmp_path / name)
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-Wall", "-Werror", *flags, "-D__HIP_PLATFORM_AMD__",
           f"-I{os.path.join(ROOT, 'csrc')}", f"-I{os.path.join(ROCM, 'include')}", SRC, "-o", exe,
           f"-L{os.path.join(ROCM, 'lib')}", "-lamdhip64", "-lcrypto", "-lz", "-lpthread",
           f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _run(exe, tmp_path, env_extra):
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, str(out)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "selftest ok" in r.stdout
    z = zipfile.ZipFile(out / "t.bin")
    assert z.testzip() is None
    assert [i.file_size for i in z.infolist()] == [1000, 40 << 20, 77]


def test_ckpt_engine_asan_ubsan(tmp_path):
    exe = _build(tmp_path, ["-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                            "-fno-sanitize-recover=undefined"], "selftest_asan")
    _run(exe, tmp_path, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})


def test_ckpt_engine_tsan(tmp_path):
    exe = _build(tmp_path, ["-fsanitize=thread"], "selftest_tsan")
    _run(exe, tmp_path, {"TSAN_OPTIONS": "halt_on_error=1"})
