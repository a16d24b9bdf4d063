"""Multi-process path on CPU (gloo, world_size 2): video sharding, the
max-over-ranks timing reduction and the optional gather to rank 0."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from eks_amd import dist


def test_shard_range_partitions():
    for total in (1, 7, 128, 1024, 1025):
        for world in (1, 2, 3, 8):
            spans = [dist.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and b >= a
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total_videos, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    r, w, _ = dist.init(backend="gloo")
    lo, hi = dist.shard_range(total_videos, w, r)
    # per-rank "outputs": video id in every element, shape (videos, T, K, 2)
    local = torch.arange(lo, hi, dtype=torch.float64).view(-1, 1, 1, 1).expand(-1, 5, 3, 2)
    full = dist.gather_to_rank0(local.contiguous(), total_videos)
    tmax = dist.max_over_ranks(float(r + 1))
    units = dist.sum_over_ranks(float(hi - lo))
    dist.barrier()
    if r == 0:
        q.put((full[:, 0, 0, 0].tolist(), tmax, units))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("total", [7, 16])
def test_gloo_world2_gather_and_reductions(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    ids, tmax, units = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ids == [float(v) for v in range(total)]
    assert tmax == 2.0
    assert units == float(total)
