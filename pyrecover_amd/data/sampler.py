"""Resumable, deterministic, distributed sampler.

Replaces ``DistributedSampler`` / ``shuffle=True`` of reference train.py:65-84, whose position is
never saved (resume replays the epoch from its start). This sampler's permutation is
a pure function of ``(seed, epoch)``, it is sharded ``rank::num_replicas`` exactly like
``DistributedSampler`` (padding to a multiple of the world size), and its position is explicit
state: the training loop reports consumed batches, ``state_dict()`` returns
``{epoch, cursor, seed, ...}`` and ``load_state_dict`` resumes mid-epoch. It exposes ``set_state``
so the reference-compatible checkpoint code stores it under the same ``sampler_state`` key
(reference pyrecover/checkpoint.py:72-73).
"""
from __future__ import annotations

import math
from typing import Iterator

import torch
from torch.utils.data import Sampler


class ResumableDistributedSampler(Sampler[int]):
    def __init__(self, dataset_len: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.dataset_len = dataset_len
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        self.cursor = 0  # samples of this rank's shard already consumed in `epoch`
        if drop_last and dataset_len % num_replicas:
            self.num_samples = dataset_len // num_replicas
        else:
            self.num_samples = math.ceil(dataset_len / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def _indices(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.dataset_len, generator=g).tolist()
        else:
            idx = list(range(self.dataset_len))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad > 0:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        return idx[self.rank:self.total_size:self.num_replicas]

    def __iter__(self) -> Iterator[int]:
        return iter(self._indices()[self.cursor:])

    def __len__(self) -> int:
        return self.num_samples - self.cursor

    def set_epoch(self, epoch: int):
        if epoch != self.epoch:
            self.epoch = epoch
            self.cursor = 0

    def advance(self, n_samples: int):
        """Record that the trainer consumed n samples of this rank's shard."""
        self.cursor += n_samples

    def state_dict(self):
        return {"epoch": self.epoch, "cursor": self.cursor, "seed": self.seed, "shuffle": self.shuffle,
                "num_replicas": self.num_replicas, "rank": self.rank, "dataset_len": self.dataset_len}

    def load_state_dict(self, sd):
        if sd.get("num_replicas", self.num_replicas) != self.num_replicas:
            # world size changed: keep the epoch, restart its shard deterministically at the same
            # global sample offset (cursor scaled by the world-size ratio)
            consumed_global = int(sd["cursor"]) * int(sd["num_replicas"])
            self.cursor = consumed_global // self.num_replicas
        else:
            self.cursor = int(sd["cursor"])
        self.epoch = int(sd["epoch"])
        self.seed = int(sd.get("seed", self.seed))
        self.shuffle = bool(sd.get("shuffle", self.shuffle))

    set_state = load_state_dict
