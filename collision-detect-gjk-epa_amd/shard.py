"""Multi-rank driver over the library's multi-GPU entries (one process per GPU, SURVEY.md §8 row e).

Pairs are independent, so a job of P pairs splits into contiguous shards (gjkepa_shard_range) with
no data-path exchange; the only collective is the all-gather of fixed-size contact records (config
C3), done by the library's RCCL communicator (gjkepa_comm_* / gjkepa_allgather_records_device) over
xGMI.  torch.distributed is the control plane only: it broadcasts the RCCL unique id, runs barriers
and reduces timings.  The gloo path (host-staged gather) is the CPU / one-GPU rehearsal.
"""
from __future__ import annotations

import gjkepa


def shard_range(total_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """[first, first + count) of the pair list owned by `rank` (gjkepa_shard_range)."""
    if world < 1 or not 0 <= rank < world or total_pairs < 0:
        raise ValueError("bad shard arguments")
    return gjkepa.shard_range(total_pairs, world, rank)


def make_comm(world: int, rank: int, device: int, group=None) -> gjkepa.Comm:
    """The library's RCCL communicator; rank 0's unique id travels over torch.distributed."""
    import torch.distributed as dist

    box = [gjkepa.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    return gjkepa.Comm(world, rank, box[0], device)


def allgather_records(local, world: int, group=None):
    """All-gather equal-size uint8 record shards (CPU torch tensors, gloo) into rank order."""
    import torch
    import torch.distributed as dist

    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out


class RecordExchange:
    """Per-step all-gather of a rank's contact records (config C3's exchange).

    `buffer()` returns the record buffer the next step fills (a view of this rank's slot inside the
    gathered buffer, so the gather runs in place); `submit(stream)` all-gathers it, in rank order.
    With a library communicator (`comm`, RCCL) `nbuf` buffers rotate and each gather runs on its own
    HIP stream after the compute stream's kernels, overlapping the next step's kernels; `buffer()`
    makes the compute stream wait for that buffer's previous gather.  Without one (gloo rehearsal)
    the records are gathered through host memory, in line.  `drain()` waits for every gather."""

    def __init__(self, nbytes: int, world: int, rank: int, device, precision: int, comm: gjkepa.Comm | None = None,
                 nbuf: int = 2, group=None, device_group=None):
        import torch

        self.world, self.rank, self.group, self.comm = world, rank, group, comm
        # device_group: a torch.distributed "nccl" (RCCL) process group, the device-to-device exchange when
        # the library's communicator is not available (same overlapped, double-buffered schedule)
        self.device_group = device_group if comm is None else None
        self.precision = precision
        self.nbytes = nbytes
        self.count = nbytes // gjkepa.load().gjkepa_record_bytes(precision)
        k = nbuf if self.overlap else 1
        self.gathered = [torch.zeros(world * nbytes, dtype=torch.uint8, device=device) for _ in range(k)]
        self.local = [g[rank * nbytes:(rank + 1) * nbytes] for g in self.gathered]
        self.stream = torch.cuda.Stream(device=device) if self.overlap else None
        self.done = [None] * k
        self.steps = 0
        self.cur = 0

    @property
    def overlap(self) -> bool:
        return self.comm is not None or self.device_group is not None

    def buffer(self, stream=None):
        b = self.steps % len(self.local)
        if self.done[b] is not None and stream is not None:
            stream.wait_event(self.done[b])      # the gather that read this buffer has finished
        self.cur = b
        return self.local[b]

    def submit(self, stream=None) -> None:
        import torch
        import torch.distributed as dist

        b = self.cur
        self.steps += 1
        if not self.overlap:                    # gloo rehearsal: host-staged
            g = torch.empty(self.gathered[b].numel(), dtype=torch.uint8)
            dist.all_gather_into_tensor(g, self.local[b].cpu(), group=self.group)
            self.gathered[b].copy_(g)
            return
        ready = torch.cuda.Event()
        ready.record(stream)
        self.stream.wait_event(ready)
        if self.comm is not None:
            self.comm.allgather_records(self.precision, self.local[b].data_ptr(), self.gathered[b].data_ptr(),
                                        self.count, self.stream.cuda_stream)
        else:
            with torch.cuda.stream(self.stream):
                dist.all_gather_into_tensor(self.gathered[b], self.local[b], group=self.device_group)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.done[b] = ev

    def drain(self) -> None:
        for k, ev in enumerate(self.done):
            if ev is not None:
                ev.synchronize()
                self.done[k] = None

    @property
    def last(self):
        """The records of the most recent step (this rank's shard)."""
        return self.local[(self.steps - 1) % len(self.local)]

    @property
    def last_gathered(self):
        """Every rank's records of the most recent step, in rank order."""
        return self.gathered[(self.steps - 1) % len(self.gathered)]
