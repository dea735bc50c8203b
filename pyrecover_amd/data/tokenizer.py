"""Tokenizer loading with an offline fallback.

The reference calls ``AutoTokenizer.from_pretrained(args.tokenizer_name_or_path)`` (reference
train.py:54), which needs the HF hub. Here we try a local/cached HF tokenizer first
(``local_files_only``) and otherwise fall back to :class:`ByteTokenizer`, a dependency-free
byte-level tokenizer with the same ``encode_plus`` / ``pad_token_id`` / ``vocab_size`` surface.
"""
from __future__ import annotations

import logging
from typing import Dict, List

logger = logging.getLogger("pyrecover")


class ByteTokenizer:
    """UTF-8 bytes -> ids 3..258; 0 = pad, 1 = bos, 2 = eos."""

    pad_token_id = 0
    bos_token_id = 1
    eos_token_id = 2

    def __init__(self, vocab_size: int = 259):
        if vocab_size < 259:
            raise ValueError("ByteTokenizer needs vocab_size >= 259")
        self.vocab_size = vocab_size

    def encode(self, text: str) -> List[int]:
        return [self.bos_token_id] + [b + 3 for b in text.encode("utf-8", errors="replace")]

    def encode_plus(self, text: str, max_length: int, padding: str = "max_length", truncation: bool = True,
                    padding_side: str = "right", **_) -> Dict[str, List[int]]:
        ids = self.encode(text)
        if truncation:
            ids = ids[:max_length]
        n = len(ids)
        if padding == "max_length" and n < max_length:
            pad = [self.pad_token_id] * (max_length - n)
            ids = ids + pad if padding_side == "right" else pad + ids
        mask = [1 if i < n else 0 for i in range(len(ids))] if padding_side == "right" else \
            [0] * (len(ids) - n) + [1] * n
        return {"input_ids": ids, "attention_mask": mask}

    def __call__(self, text, **kw):
        return self.encode_plus(text, **kw)


def load_tokenizer(name_or_path: str):
    try:
        from transformers import AutoTokenizer

        tok = AutoTokenizer.from_pretrained(name_or_path, local_files_only=True)
        if tok.pad_token_id is None:
            tok.pad_token = tok.eos_token
        return tok
    except Exception as e:  # no network / not cached
        logger.warning(f"tokenizer {name_or_path!r} unavailable offline ({type(e).__name__}); using ByteTokenizer")
        return ByteTokenizer()
