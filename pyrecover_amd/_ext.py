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
    env = _attn_env()  # a malformed PYRECOVER_ATTN_BWD_FUSED raises ValueError naming it, not a load error
    try:
        import torch  # noqa: F401  (loads torch's HIP runtime first; our .so binds to it)
        from pyrecover_amd import _C as mod
    except BaseException as e:  # pragma: no cover - exercised only when the build is missing
        _err = e
        raise RuntimeError(
            "pyrecover_amd native extension is not built or failed to load "
            f"({e!r}). Build it with `python -m pyrecover_amd._build` (hipcc --offload-arch=gfx950)."
        ) from e
    _apply_options(mod, env)
    _C = mod  # published only once the options applied
    return _C


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


# Attention kernel selection (csrc/kernels/attention.hip AttnOptions): -1 = by shape. The launchers
# read no environment. set_attn_options() changes the options between launches (tests, A/B tools);
# of the environment only PYRECOVER_ATTN_BWD_FUSED (the one experimental kernel path: the fused
# deterministic backward) is read, once, when the extension loads -- every other option is a
# measured by-shape default (docs/KNOBS.md).
# *_order: block order of the forward / dQ / dK/dV grids (attention.hip block_tile): -1 = XCD-grouped
# by shape, 0 = heavy tiles first across the grid, G = XCD-grouped with G heads per group.
_ATTN_DEFAULTS = {"fwd_pipe": -1, "fwd_thr": 8.0, "dkdv_impl": -1, "dq_pipe": -1, "dkdv_split": 1, "dkdv_kreg": -2,
                  "bwd_fused": 0, "bwd_window": -1, "fwd_order": -1, "dq_order": -1, "dkdv_order": -1,
                  }
_ATTN_ENV = ("bwd_fused",)
_attn_opts = dict(_ATTN_DEFAULTS)


def _attn_env() -> dict:
    env = {}
    for key in _ATTN_ENV:
        name = "PYRECOVER_ATTN_" + key.upper()
        v = os.environ.get(name)
        if v is not None and v != "":
            try:
                env[key] = int(v)
            except ValueError:
                raise ValueError(f"{name}={v!r} is not a valid int") from None
    # PYRECOVER_ATTN_BWD_FUSED=1 selects the fused backward by shape: only where its grid (one
    # workgroup per batch x kv head) fills the chip. At batch 1 (8 workgroups for Llama-3-8B) it was
    # 78% slower, so it never runs there (round-5 verdict). set_attn_options(bwd_fused=1) still
    # forces it at every shape (kernel tests).
    if env.get("bwd_fused") == 1:
        env["bwd_fused"] = -1
    return env


def _apply_options(mod, env: dict) -> None:
    opts = dict(_attn_opts)
    opts.update(env)
    mod.attn_set_options(opts["fwd_pipe"], opts["fwd_thr"], opts["dkdv_impl"], opts["dq_pipe"], opts["dkdv_split"],
                         opts["dkdv_kreg"], opts["bwd_fused"], opts["bwd_window"])
    mod.attn_set_order(opts["fwd_order"], opts["dq_order"], opts["dkdv_order"])
    _attn_opts.update(opts)


def set_attn_options(**kw) -> dict:
    """Set attention kernel selection knobs (fwd_pipe, fwd_thr, dkdv_impl, dq_pipe, dkdv_split, dkdv_kreg,
    bwd_fused, bwd_window, fwd_order, dq_order, dkdv_order); keys left out
    keep their value, ``None`` restores the default. Returns the previous settings."""
    mod = native()  # loads the extension and applies PYRECOVER_ATTN_BWD_FUSED first
    prev = dict(_attn_opts)
    new = {}
    for k, v in kw.items():
        if k not in _ATTN_DEFAULTS:
            raise KeyError(f"unknown attention option {k!r}")
        new[k] = _ATTN_DEFAULTS[k] if v is None else type(_ATTN_DEFAULTS[k])(v)
    _apply_options(mod, new)
    return prev
