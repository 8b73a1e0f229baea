"""Pair-list sharding across ranks (one process per GPU) and the contact all-gather.

Pairs are independent, so a job of P pairs splits into contiguous shards with no data-path
exchange; the only collective is the all-gather of fixed-size contact records (RCCL over xGMI on
MI355X, gloo in the CPU tests) when every rank needs every contact (config C3).
"""
from __future__ import annotations


def shard_range(total_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """[first, first + count) of the pair list owned by `rank`; shards differ by at most one pair."""
    if world < 1 or not 0 <= rank < world or total_pairs < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total_pairs, world)
    first = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return first, count


def allgather_records(local, world: int, group=None):
    """All-gather equal-size uint8 record shards (torch tensors) into rank order.
    `local` must hold the same number of bytes on every rank (use equal shards)."""
    import torch
    import torch.distributed as dist

    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out


class RecordExchange:
    """Per-step all-gather of a rank's contact records (config C3's exchange).

    `buffer()` returns the record buffer the next step fills; `submit()` all-gathers it, in rank
    order, into `gathered[b]`.  With `overlap` (the RCCL path) `nbuf` buffers rotate and the gather
    is asynchronous: it runs on the collective's own stream while the next step's kernels fill the
    next buffer, and `buffer()` makes the compute stream wait for a buffer's previous gather before
    handing it out again.  `host_staged` (gloo rehearsal on one GPU) copies through host memory and
    gathers in line.  `drain()` waits for every outstanding gather."""

    def __init__(self, nbytes: int, world: int, device, overlap: bool = False, host_staged: bool = False,
                 nbuf: int = 2, group=None):
        import torch

        self.world, self.group, self.host_staged = world, group, host_staged
        self.overlap = overlap and not host_staged
        k = nbuf if self.overlap else 1
        self.local = [torch.zeros(nbytes, dtype=torch.uint8, device=device) for _ in range(k)]
        self.gathered = [torch.empty(world * nbytes, dtype=torch.uint8, device=device) for _ in range(k)]
        self.works = [None] * k
        self.steps = 0
        self.cur = 0

    def buffer(self):
        b = self.steps % len(self.local)
        if self.works[b] is not None:
            self.works[b].wait()        # the gather that read this buffer has finished
            self.works[b] = None
        self.cur = b
        return self.local[b]

    def submit(self) -> None:
        import torch
        import torch.distributed as dist

        b = self.cur
        self.steps += 1
        if self.host_staged:
            g = torch.empty(self.gathered[b].numel(), dtype=torch.uint8)
            dist.all_gather_into_tensor(g, self.local[b].cpu(), group=self.group)
            self.gathered[b].copy_(g)
        elif self.overlap:
            self.works[b] = dist.all_gather_into_tensor(self.gathered[b], self.local[b], group=self.group,
                                                        async_op=True)
        else:
            dist.all_gather_into_tensor(self.gathered[b], self.local[b], group=self.group)

    def drain(self) -> None:
        for k, w in enumerate(self.works):
            if w is not None:
                w.wait()
                self.works[k] = None

    @property
    def last(self):
        """The records of the most recent step (this rank's shard)."""
        return self.local[(self.steps - 1) % len(self.local)]

    @property
    def last_gathered(self):
        """Every rank's records of the most recent step, in rank order."""
        return self.gathered[(self.steps - 1) % len(self.gathered)]
