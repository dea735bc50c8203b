"""Hot-path ops: HIP kernels (gfx950) for GPU tensors, reference torch math for CPU tensors."""
from .fused import (  # noqa: F401
    FlatSlotAdapter,
    UnflatSlot,
    add_layer_norm,
    add_rms_norm,
    attention_block,
    embedding,
    flash_attention,
    linear_cross_entropy,
    swiglu_mlp,
)
from .reference import (  # noqa: F401
    apply_rotary_emb_ref,
    attention_ref,
    cross_entropy_ref,
    precompute_freqs_cis,
    rmsnorm_ref,
    rope_table,
)
