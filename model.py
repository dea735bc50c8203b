"""Reference-compatible module path (reference model.py): ``from model import Transformer,
TransformerModelArgs`` keeps working; the implementation is pyrecover_amd's fused-kernel model."""
from pyrecover_amd.config import TransformerModelArgs  # noqa: F401
from pyrecover_amd.models.llama import (  # noqa: F401
    Attention,
    FeedForward,
    RMSNorm,
    Transformer,
    TransformerBlock,
)
from pyrecover_amd.ops.reference import apply_rotary_emb_ref as apply_rotary_emb  # noqa: F401
from pyrecover_amd.ops.reference import precompute_freqs_cis  # noqa: F401
