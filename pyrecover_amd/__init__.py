"""pyrecover_amd: MI355X-native (gfx950) DDP training + checkpointing engine with PyRecover's
capabilities. Hot path = hand-written HIP kernels (pyrecover_amd._C), gradients over RCCL/xGMI,
checkpoint I/O through a native async engine."""

__version__ = "0.1.0"
