"""Direct intra-node all-reduce over xGMI for the flat gradient buffer.

RCCL's ring moves every byte around the 8 GPUs over one link per direction per ring. On an MI355X
node every GPU has a direct xGMI link to each of its 7 peers, so this backend works per link
instead. Default engine (``csrc/dist/xgmi.cpp`` XgmiEngine, native):

* reduce-scatter: rank r owns slice r of each bucket; ONE pull-reduce kernel reads slice r from
  every rank's IPC-mapped gradient buffer (the 7 peers' over their xGMI links at once) and sums them
  in fp32 in rank order into its own buffer: one rounding, so every rank gets bit-identical values,
  deterministically, and no staging copy;
* all-gather: ONE pull-gather kernel copies every owner's reduced slice into this rank's buffer;
* both kernels run on one high-priority comm stream, scheduled by a C++ worker thread, so the
  backward thread only records an event and enqueues the bucket (no Python in the critical window,
  one hardware queue for all of it).

Per bucket, the traffic per link is bucket/W per phase. (Round 4's copy-engine path -- one copy
stream per peer into local staging, then the reduction kernel, orchestrated by a Python thread -- was
replaced by this engine and removed in round 6.)

Cross-process ordering uses interprocess HIP events only: a rank's comm stream waits, on the GPU,
on its peers' "bucket ready" / "slice reduced" events, and no kernel spins. The host only
guarantees that an event was recorded (for THIS step) before anyone waits on it: every rank
publishes a per-bucket sequence number in a page of host shared memory right after recording, and
the worker of a peer polls that word (microseconds). The backward thread never blocks.

The gradient buffer is reallocated with ``hipMalloc`` so it can be exported with
``hipIpcGetMemHandle``. Opt-in: ``GradReducer(..., backend="xgmi")``, ``train.py --allreduce
xgmi``, ``bench.py --allreduce xgmi``. RCCL stays the default.
"""
from __future__ import annotations

import os
import time
import uuid
from multiprocessing import shared_memory
from typing import List, Sequence, Tuple

import numpy as np

import torch
import torch.distributed as dist

from .. import _ext



def _device_identity(i: int) -> str:
    """Stable identity of visible device i across processes (UUID, else PCI address)."""
    p = torch.cuda.get_device_properties(i)
    u = getattr(p, "uuid", None)
    if u is not None and str(u).strip("0-") != "":
        return str(u)
    pci = tuple(getattr(p, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if any(x is not None for x in pci):
        return "pci:%s:%s:%s" % pci
    return f"{p.name}#{i}"


def _hidden_ranks(vis) -> List[int]:
    """Ranks whose GPU some rank cannot see; vis[r] = (rank r's device identity, identities rank r sees)."""
    return sorted({r for r, (own, _) in enumerate(vis) for _, seen in vis if own not in seen})

class _Work:
    __slots__ = ("owner", "b", "seq")

    def __init__(self, owner, b):
        self.owner = owner
        self.b = b
        self.seq = 0  # the step this bucket belongs to (a ticket for wait)

    def wait(self):
        """Current stream waits (GPU-side) for the all-reduced bucket."""
        self.owner.eng.wait(self.b, self.seq, torch.cuda.current_stream(self.owner.dev).cuda_stream)


class _HostSeq:
    """[world, slots] int64 sequence words in one POSIX shared-memory page set (node-local ranks):
    rank r publishes ``seq`` in its own row; readers poll a peer's word until it reaches ``seq``.
    Aligned 8-byte stores/loads are single-copy atomic on x86-64."""

    def __init__(self, rank: int, world: int, slots: int, group):
        name = [f"pra_xgmi_{uuid.uuid4().hex[:16]}" if rank == 0 else None]
        dist.broadcast_object_list(name, src=0, group=group)
        size = world * slots * 8
        self.owner = rank == 0
        if self.owner:
            self.shm = shared_memory.SharedMemory(name=name[0], create=True, size=size)
        dist.barrier(group=group)
        if not self.owner:
            self.shm = shared_memory.SharedMemory(name=name[0], create=False, size=size)
            # Python < 3.13 registers attached segments with the resource tracker too, which would
            # unlink rank 0's segment when this process exits; only the creator owns it
            from multiprocessing import resource_tracker

            resource_tracker.unregister(self.shm._name, "shared_memory")
        else:
            import atexit

            atexit.register(self.close)  # never leave the page behind in /dev/shm
        self.a = np.ndarray((world, slots), dtype=np.int64, buffer=self.shm.buf)
        if self.owner:
            self.a[:] = 0
        dist.barrier(group=group)
        self.rank = rank

    def publish(self, slot: int, seq: int):
        self.a[self.rank, slot] = seq

    def wait(self, r: int, slot: int, seq: int, timeout: float = 600.0):
        """Poll rank r's word until it reaches seq (the host side of the engine's wait_word)."""
        if self.a[r, slot] >= seq:
            return
        t0 = time.perf_counter()
        spins = 0
        while self.a[r, slot] < seq:
            spins += 1
            if spins > 200:
                time.sleep(20e-6)
            if time.perf_counter() - t0 > timeout:
                raise TimeoutError(f"xgmi: rank {r} did not publish slot {slot} seq {seq}")

    def address(self) -> int:
        """Base address of the [world, slots] int64 words in this process (for the native engine)."""
        return self.a.ctypes.data

    def close(self):
        if getattr(self, "a", None) is None:
            return
        self.a = None
        self.shm.close()
        if self.owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass


class XgmiAllReduce:
    def __init__(self, flat, ranges: Sequence[Tuple[int, int]], group=None):
        self.C = _ext.native().xgmi
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = W = dist.get_world_size(group)
        if not 1 < W <= 16:
            raise ValueError("xgmi all-reduce needs 2..16 ranks on one node")
        self.flat = flat
        self.dev = flat.grad.device
        di = self.dev.index
        self.dtype = flat.grad.dtype
        self.esz = flat.grad.element_size()
        # 1) CPU barriers for the comm thread (its own gloo group, used by nothing else)
        self.hgroup = dist.new_group(backend="gloo")
        # 2) every peer GPU must be visible to map its buffer: under SLURM per-task isolation
        # (--gpus-per-task=1 / --gpu-bind) each rank sees only its own device and peer IPC cannot
        # work. Devices are compared by identity (UUID / PCI address), not by index, so ranks that
        # share one GPU (one-GPU rehearsals) pass and isolated ranks that all see "device 0" do not.
        # Decided collectively, so every rank raises instead of one rank hanging the others.
        n_vis = torch.cuda.device_count()
        mine = (_device_identity(di), [_device_identity(i) for i in range(n_vis)])
        vis: List = [None] * W
        dist.all_gather_object(vis, mine, group=self.hgroup)
        hidden = _hidden_ranks(vis)
        if hidden:
            raise RuntimeError(
                f"xgmi all-reduce needs every rank's GPU visible to every rank (GPUs of ranks {hidden} are "
                f"hidden from some peers; visible per rank: {[len(s) for _, s in vis]}); per-task GPU "
                "isolation (srun --gpus-per-task=1 / --gpu-bind, or per-rank ROCR_VISIBLE_DEVICES) hides "
                "the peers. Use the default RCCL all-reduce (--allreduce rccl) or launch with every GPU "
                "visible.")
        # 3) exportable gradient buffer
        buf = self.C.ipc_empty(flat.grad.numel(), self.dtype, di)
        buf.copy_(flat.grad)
        flat.rebind_grad(buf)
        self.buf = buf
        # 4) peer buffers (a failed open is reported on every rank)
        handles: List = [None] * W
        dist.all_gather_object(handles, self.C.ipc_mem_handle(buf), group=self.hgroup)
        base = buf.data_ptr()
        self.peer_base, err = [], None
        for r in range(W):
            if r == self.rank:
                self.peer_base.append(base)
                continue
            try:
                self.peer_base.append(self.C.ipc_open_mem(handles[r], di))
            except RuntimeError as e:  # noqa: PERF203
                err = f"rank {self.rank}: ipc_open_mem of rank {r}'s buffer failed: {e}"
                break
        errs: List = [None] * W
        dist.all_gather_object(errs, err, group=self.hgroup)
        bad = [e for e in errs if e]
        if bad:
            raise RuntimeError("xgmi all-reduce cannot map peer gradient buffers (GPU isolation or no "
                               "dmabuf IPC; HSA_ENABLE_IPC_MODE_LEGACY=0 is required): " + "; ".join(bad))
        # 4) slices (identical on every rank; 8-element = 16-B aligned boundaries)
        self.ranges = list(ranges)
        self.slices = []
        for lo, hi in self.ranges:
            n = hi - lo
            cuts = [lo + ((n * r // W) // 8) * 8 for r in range(W)] + [hi]
            self.slices.append([(cuts[r], cuts[r + 1]) for r in range(W)])
        # 5) events: per bucket "ready" and "reduced" (interprocess), one per-step "done"
        nb = len(self.ranges)
        self.ev_ready = [self.C.ipc_event_create(di) for _ in range(nb)]
        self.ev_rs = [self.C.ipc_event_create(di) for _ in range(nb)]
        self.ev_step = self.C.ipc_event_create(di)
        mine = ([self.C.ipc_event_handle(e) for e in self.ev_ready], [self.C.ipc_event_handle(e) for e in self.ev_rs],
                self.C.ipc_event_handle(self.ev_step))
        allh: List = [None] * W
        dist.all_gather_object(allh, mine, group=self.hgroup)
        self.peer_ready, self.peer_rs, self.peer_step = [], [], []
        for r in range(W):
            if r == self.rank:
                self.peer_ready.append(self.ev_ready)
                self.peer_rs.append(self.ev_rs)
                self.peer_step.append(self.ev_step)
            else:
                self.peer_ready.append([self.C.ipc_event_open(h, di) for h in allh[r][0]])
                self.peer_rs.append([self.C.ipc_event_open(h, di) for h in allh[r][1]])
                self.peer_step.append(self.C.ipc_event_open(allh[r][2], di))
        # 6) host sequence words: [ready b | reduced b | step]
        self.nb = nb
        self.seq = 1  # current step's sequence number (published values start at 1)
        self.hseq = _HostSeq(self.rank, W, 2 * nb + 1, self.hgroup)
        # the native engine (csrc/dist/xgmi.cpp XgmiEngine): one comm stream, one pull-reduce kernel
        # reading every peer's slice over xGMI and one pull-gather kernel per bucket, scheduled by a
        # C++ worker thread
        code = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[self.dtype]
        cuts = [c for sl in self.slices for c in [s0 for s0, _ in sl] + [sl[-1][1]]]
        self.eng = self.C.XgmiEngine(
            di, self.rank, W, code, self.esz, list(self.peer_base), cuts, self.hseq.address(),
            list(self.ev_ready), list(self.ev_rs), self.ev_step,
            [e for r in range(W) for e in self.peer_ready[r]], [e for r in range(W) for e in self.peer_rs[r]],
            list(self.peer_step))
        dist.barrier(group=self.hgroup)

    # --- backward thread -----------------------------------------------------------------
    def launch(self, b: int) -> _Work:
        w = _Work(self, b)
        w.seq = self.eng.launch(b, torch.cuda.current_stream(self.dev).cuda_stream)
        return w

    def end_step(self):
        """After every bucket of the step was waited on: no rank may overwrite its gradient
        buffer (next backward) before every peer finished reading it."""
        self.eng.end_step(torch.cuda.current_stream(self.dev).cuda_stream)
        self.seq += 1
