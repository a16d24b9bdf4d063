"""Multi-GPU plumbing: one process per GPU, trajectories sharded by video.

Videos (and therefore their keypoint trajectories) are independent, so the
smoother needs no collective on its data path.  Each
rank smooths a contiguous block of videos and keeps its outputs resident;
``gather_to_rank0`` is the optional single RCCL gather of the (videos, T, K,
2) float64 results over xGMI for callers that want everything on one rank.
The timing reduction (max over ranks) is the only collective ``bench.py``
issues.  All of this runs unchanged on ``gloo`` (CPU tests) and ``nccl``
(= RCCL on ROCm).
"""
from __future__ import annotations

import os


def env_world():
    """(rank, world_size, local_rank) from torchrun's environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_range(total: int, world: int, rank: int):
    """Contiguous block [lo, hi) of ``total`` items for ``rank``; the first
    ``total % world`` ranks get one extra item."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def init(backend: str | None = None, force: bool = False):
    """Initialise torch.distributed when WORLD_SIZE > 1 (or ``force``: a
    one-rank group, e.g. to run the RCCL code paths on one GPU), 127.0.0.1
    rendezvous from torchrun's MASTER_ADDR/PORT.  With nccl (= RCCL) the rank
    is bound to its GPU (LOCAL_RANK) before the group is created and the
    device is handed to the group (``device_id``), so the communicator and
    every barrier use that device instead of a guess."""
    import torch.distributed as dist
    rank, world, local = env_world()
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import torch
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def max_over_ranks(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_to_rank0(local, total_rows: int):
    """Gather every rank's (rows_r, ...) shard into one (total_rows, ...)
    tensor on rank 0 (uneven shards allowed: shards are padded to the
    largest one for the collective).  Returns the tensor on rank 0, None
    elsewhere.  One collective; on ROCm with backend nccl this is RCCL over
    xGMI."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return local
    rank, world = dist.get_rank(), dist.get_world_size()
    if local.is_cuda and dist.get_backend() == "gloo":
        # gloo gathers host tensors (the CPU tests and the 1-GPU rehearsal)
        full = gather_to_rank0(local.cpu(), total_rows)
        return None if full is None else full.to(local.device)
    sizes = [shard_range(total_rows, world, r) for r in range(world)]
    rows = [hi - lo for lo, hi in sizes]
    cap = max(rows)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, gather_list=bufs, dst=0)
    if rank != 0:
        return None
    return torch.cat([b[:n] for b, n in zip(bufs, rows)], dim=0)
