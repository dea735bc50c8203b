"""Loader for the in-tree native extension ``pyrecover_amd._C``.

On a GPU box the HIP path is mandatory: if the extension is missing or fails to import while a
GPU tensor reaches an op, we raise instead of silently falling back to PyTorch math. The CPU
(reference-math) path exists only for CPU/gloo runs and as the numerics oracle in tests.
"""
from __future__ import annotations

import os

_C = None
_err: BaseException | None = None


def native():
    """Return the native module, importing it on first use (raises if unavailable)."""
    global _C, _err
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (loads torch's HIP runtime first; our .so binds to it)
        from pyrecover_amd import _C as mod
        _C = mod
        return _C
    except BaseException as e:  # pragma: no cover - exercised only when the build is missing
        _err = e
        raise RuntimeError(
            "pyrecover_amd native extension is not built or failed to load "
            f"({e!r}). Build it with `python -m pyrecover_amd._build` (hipcc --offload-arch=gfx950)."
        ) from e


def available() -> bool:
    try:
        native()
        return True
    except RuntimeError:
        return False


def require_for(t) -> object:
    """Native module for a GPU tensor; raises loudly if the HIP build is absent."""
    if os.environ.get("PYRECOVER_AMD_FORCE_REFERENCE") == "1":
        raise RuntimeError("PYRECOVER_AMD_FORCE_REFERENCE=1 is set but a GPU tensor reached a native op")
    return native()


# dtypes the HIP kernels are instantiated for. GPU tensors of other dtypes (fp64) run the
# plain-torch math of pyrecover_amd.ops.reference on the GPU, as do attention and the
# transposing kernels for fp32 (their MFMA tiles are 16-bit).
def hip(t) -> bool:
    """True when ``t`` is a GPU tensor whose dtype the element-wise HIP kernels take (bf16/fp16/fp32)."""
    import torch

    return t.is_cuda and t.dtype in (torch.bfloat16, torch.float16, torch.float32)


def hip16(t) -> bool:
    """True for GPU bf16/fp16 tensors (the MFMA attention and the transposing kernels)."""
    import torch

    return t.is_cuda and t.dtype in (torch.bfloat16, torch.float16)
