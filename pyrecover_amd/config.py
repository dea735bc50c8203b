"""Model configuration and named presets.

``TransformerModelArgs`` keeps the field names and defaults of the reference dataclass
(reference model.py:9-22) so existing code constructing it keeps working; presets add the
shapes named in BASELINE.json (GPT-2-small/medium-shape, Llama-2-7B-shape, Llama-3-8B-shape).
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional


@dataclass
class TransformerModelArgs:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: Optional[int] = None
    multiple_of: int = 256  # make SwiGLU hidden layer size multiple of large power of 2
    ffn_dim_multiplier: Optional[float] = None
    norm_eps: float = 1e-5
    rope_theta: float = 10000
    norm_type: str = "rmsnorm"
    seq_len: int = 2048
    vocab_size: int = -1
    use_flash_attention: bool = False

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @property
    def kv_heads(self) -> int:
        return self.n_heads if self.n_kv_heads is None else self.n_kv_heads

    @property
    def ffn_hidden(self) -> int:
        """SwiGLU hidden size, same rounding as reference model.py:258-262."""
        hidden = int(2 * (4 * self.dim) / 3)
        if self.ffn_dim_multiplier is not None:
            hidden = int(self.ffn_dim_multiplier * hidden)
        return self.multiple_of * ((hidden + self.multiple_of - 1) // self.multiple_of)


# The reference hard-codes this architecture in train.py:88-99 (vocab from the
# Mistral-Nemo tokenizer = 131072).
PRESETS = {
    "llama3-8b": TransformerModelArgs(dim=4096, n_layers=32, n_heads=32, n_kv_heads=8, ffn_dim_multiplier=1.3,
                                      multiple_of=1024, rope_theta=500000, vocab_size=131072),
    "llama2-7b": TransformerModelArgs(dim=4096, n_layers=32, n_heads=32, n_kv_heads=32, multiple_of=256,
                                      rope_theta=10000, vocab_size=32000),
    # GPT-2 shapes (dims/heads/vocab padded to 50304) with LayerNorm; the block structure stays
    # the reference's (RoPE, SwiGLU, untied head) -- "shape", as BASELINE.json configs 1-2 say.
    "gpt2-medium": TransformerModelArgs(dim=1024, n_layers=24, n_heads=16, n_kv_heads=16, multiple_of=256,
                                        vocab_size=50304, norm_type="layernorm"),
    "gpt2-small": TransformerModelArgs(dim=768, n_layers=12, n_heads=12, n_kv_heads=12, multiple_of=256,
                                       vocab_size=50304, norm_type="layernorm"),
    "llama-tiny": TransformerModelArgs(dim=256, n_layers=2, n_heads=4, n_kv_heads=2, multiple_of=64,
                                       vocab_size=512, rope_theta=10000),
    "llama-micro": TransformerModelArgs(dim=128, n_layers=2, n_heads=2, n_kv_heads=1, multiple_of=64,
                                        vocab_size=256, rope_theta=10000),
}


def get_preset(name: str, **overrides) -> TransformerModelArgs:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; choose from {sorted(PRESETS)}")
    return replace(PRESETS[name], **{k: v for k, v in overrides.items() if v is not None})
