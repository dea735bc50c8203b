"""Datasets and collator (reference dataset.py:10-61) plus synthetic data for benchmarks.

* :class:`ParquetDataset` keeps the reference semantics: memory-mapped parquet with a ``text``
  column, virtual length = ``training_samples``, sample ``idx`` tokenizes ``text[idx % rows]`` with
  right padding / truncation to ``sequence_length + 1``.
* :class:`CollatorForCLM` returns ``(inputs, labels)`` with pad labels set to -100.
* :class:`SyntheticTokenDataset` yields deterministic random token rows (a function of
  ``(seed, idx)`` only, so resuming at any sample reproduces the same stream).
* :func:`make_synthetic_parquet` writes a parquet file of random text for end-to-end runs without
  the reference's cluster dataset.
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass
from typing import Dict, List

import numpy as np
import torch
from torch.utils.data import Dataset


class ParquetDataset(Dataset):
    def __init__(self, parquet_file: str, tokenizer, sequence_length: int, training_samples: int):
        import pyarrow.parquet as pq

        self.parquet_ds = pq.read_table(parquet_file, memory_map=True)
        self.real_length = len(self.parquet_ds)
        if self.real_length == 0:
            raise ValueError(f"{parquet_file} has no rows")
        self.texts = self.parquet_ds.column("text")
        self.tokenizer = tokenizer
        self.sequence_length = sequence_length
        self.training_samples = training_samples

    def __len__(self):
        return self.training_samples

    def __getitem__(self, idx: int):
        sample_str = str(self.texts[idx % self.real_length])
        return self.tokenizer.encode_plus(sample_str, max_length=self.sequence_length + 1, padding="max_length",
                                          truncation=True, padding_side="right")


class SyntheticTokenDataset(Dataset):
    """Deterministic random token rows of length sequence_length + 1 (no pad tokens)."""

    def __init__(self, vocab_size: int, sequence_length: int, training_samples: int, seed: int = 0,
                 pad_token_id: int = 0):
        self.vocab_size = vocab_size
        self.sequence_length = sequence_length
        self.training_samples = training_samples
        self.seed = seed
        self.pad_token_id = pad_token_id

    def __len__(self):
        return self.training_samples

    def __getitem__(self, idx: int):
        rng = np.random.default_rng([self.seed, int(idx)])
        lo = 1 if self.pad_token_id == 0 else 0
        ids = rng.integers(lo, self.vocab_size, size=self.sequence_length + 1, dtype=np.int64)
        if self.pad_token_id != 0:
            ids[ids == self.pad_token_id] = (self.pad_token_id + 1) % self.vocab_size
        return {"input_ids": ids.tolist()}


@dataclass
class CollatorForCLM:
    sequence_length: int
    pad_token_id: int

    def __call__(self, examples: List[Dict[str, List[int]]]):
        input_ids = torch.as_tensor(np.asarray([e["input_ids"] for e in examples], dtype=np.int64))
        inputs = input_ids[:, :-1].clone()
        labels = input_ids[:, 1:].clone()
        labels[labels == self.pad_token_id] = -100
        assert inputs.shape[1] == labels.shape[1] == self.sequence_length
        assert inputs.shape == labels.shape
        return inputs, labels


_WORDS = ("the of and to in is was for on that with as by at from his her an were are which this be "
          "or has had not but one all their they it its been more also who would two new first after "
          "time may other some these only such when than most into over many both then use while where "
          "state city year world during later known under since made part between work").split()


def make_synthetic_parquet(path: str, n_docs: int = 256, min_words: int = 50, max_words: int = 2000,
                           seed: int = 0) -> str:
    """Write a parquet file with a ``text`` column of random word sequences."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    rnd = random.Random(seed)
    texts = [" ".join(rnd.choice(_WORDS) for _ in range(rnd.randint(min_words, max_words))) for _ in range(n_docs)]
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    pq.write_table(pa.table({"text": texts}), path)
    return path
