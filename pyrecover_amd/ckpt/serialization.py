"""torch.save-compatible archive planning without copying tensor bytes.

:func:`plan_archive` runs PyTorch's own serializer (``torch.serialization._save``: the pickle
stream, storage keys, ``.format_version``/``.storage_alignment``/``byteorder`` records) against a
recording zip writer. The result is a list of ``(record_name, host_pointer, nbytes)`` that the C++
engine (``pyrecover_amd._C.CkptEngine.write_items``) streams into a zip file. Storage payloads are
referenced by pointer (CPU tensors aliasing the pinned staging pool), so the archive is produced
with zero Python-side copies and is byte-for-byte loadable by ``torch.load`` (including
``mmap=True`` and ``weights_only=True``).
"""
from __future__ import annotations

import ctypes
import io
import pickle
import uuid
from typing import Any, List, Tuple

import torch


class _RecordingZip:
    def __init__(self, prefix: str):
        self.prefix = prefix
        self.records: List[Tuple[str, int, int]] = []
        self.keepalive: List[Any] = []

    def write_record(self, name, data, nbytes):
        full = f"{self.prefix}/{name}"
        if isinstance(data, (bytes, bytearray)):
            buf = ctypes.create_string_buffer(bytes(data), len(data))
            self.keepalive.append(buf)
            self.records.append((full, ctypes.addressof(buf), nbytes))
        elif isinstance(data, str):
            b = data.encode()
            buf = ctypes.create_string_buffer(b, len(b))
            self.keepalive.append(buf)
            self.records.append((full, ctypes.addressof(buf), len(b)))
        else:  # an UntypedStorage on the CPU
            if data.device.type != "cpu":
                raise ValueError("plan_archive: storages must be CPU (stage device tensors first)")
            self.keepalive.append(data)
            self.records.append((full, data.data_ptr(), nbytes))

    def write_record_metadata(self, name, nbytes):  # pragma: no cover - skip_data mode unused
        raise NotImplementedError


def plan_archive(obj, prefix: str = "archive"):
    """Returns (records, keepalive). Mirrors torch.save's record set and order."""
    z = _RecordingZip(prefix)
    torch.serialization._save(obj, z, pickle, 2, False)
    z.write_record("version", "3\n", 2)
    sid = str(uuid.uuid4().int)[:40].ljust(40, "0")
    z.write_record(".data/serialization_id", sid, len(sid))
    return z.records, z.keepalive


def host_view(ptr: int, nbytes: int, dtype: torch.dtype, shape) -> torch.Tensor:
    """A CPU tensor with its OWN storage aliasing host memory [ptr, ptr+nbytes) (no copy).

    Each call creates a distinct storage, so torch's serializer writes one record per tensor,
    exactly like saving independent tensors (the reference's per-parameter storages)."""
    if nbytes == 0:
        return torch.empty(shape, dtype=dtype)
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    t = torch.frombuffer(buf, dtype=torch.uint8)
    return t.view(dtype).view(shape)


def torch_save_bytes(obj) -> bytes:
    b = io.BytesIO()
    torch.save(obj, b)
    return b.getvalue()
