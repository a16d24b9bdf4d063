"""The config-4 batch job over 2 ranks sharing cuda:0 (gloo): each rank
fits and smooths its contiguous half of the videos (algo 3, the config-4
default), the outputs are gathered to rank 0 (eks_amd.dist.gather_to_rank0,
the bench's final collective) and must be BIT-identical to one process
smoothing the whole batch.  SURVEY.md §8(e) E1; bench.py --gpus N runs the
same sharding with RCCL."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

VIDEOS, K, E, T = 16, 17, 5, 10000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _smooth_videos(torch, videos):
    import bench
    from eks_amd import _lib, batch
    dev = torch.device("cuda", 0)
    obs = bench.gen_videos(torch, videos, K, E, T, 4, dev).permute(3, 0, 1, 2)
    params, _ = batch.fit(obs, kind="singleview", n=2, r=2, smooth_param=0.01, quantile_keep=25)
    flags = _lib.EKS_MODEL_A_IDENTITY | _lib.EKS_MODEL_C_IDENTITY
    out = batch.smooth(obs, params, n=2, r=2, algo=3, flags=flags, check=True)["out"]
    # (videos, T, K, 2), the layout bench.py gathers
    return out.reshape(len(videos), K, T, 2).permute(0, 2, 1, 3).contiguous()


def _worker(rank, world, port, q):
    import torch
    from eks_amd import dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    dist.init(backend="gloo")
    try:
        torch.cuda.set_device(0)
        lo, hi = dist.shard_range(VIDEOS, world, rank)
        loc = _smooth_videos(torch, range(lo, hi))
        full = dist.gather_to_rank0(loc, VIDEOS)
        if rank == 0:
            ref = _smooth_videos(torch, range(VIDEOS))
            q.put((tuple(full.shape), bool(torch.equal(full, ref)),
                   float((full - ref).abs().max())))
        dist.barrier()
    finally:
        torch.distributed.destroy_process_group()


def test_two_ranks_gathered_equal_one_rank():
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    shape, equal, diff = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert shape == (VIDEOS, T, K, 2)
    assert equal, f"sharded outputs differ from the 1-rank batch by {diff}"


def _rccl_worker(port, q):
    import torch
    from eks_amd import dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    try:
        dist.init(backend="nccl", force=True)     # RCCL, bound to cuda:0 (device_id)
        import torch.distributed as td
        backend = str(td.get_backend())
        dev = torch.device("cuda", 0)
        loc = torch.arange(3 * 5 * 2, dtype=torch.float64, device=dev).view(3, 5, 2)
        full = dist.gather_to_rank0(loc, 3)       # the padded device-tensor gather branch
        tmax = dist.max_over_ranks(2.5, device=dev)
        tsum = dist.sum_over_ranks(7.0, device=dev)
        dist.barrier()
        q.put((backend, full.is_cuda, bool(torch.equal(full, loc)), tmax, tsum))
    except Exception as exc:  # report, do not hang the parent
        q.put(("error", repr(exc)))
    finally:
        import torch.distributed as td
        if td.is_initialized():
            td.destroy_process_group()


def test_rccl_world1_collectives():
    """The nccl (= RCCL on ROCm) code paths of eks_amd.dist on one GPU: a
    world_size-1 group bound to cuda:0 runs the padded device-tensor
    gather_to_rank0 (what bench.py's N > 1 gather issues), max_over_ranks,
    sum_over_ranks and barrier through RCCL."""
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] == "nccl", res
    assert p.exitcode == 0
    _, on_gpu, equal, tmax, tsum = res
    assert on_gpu and equal
    assert tmax == 2.5 and tsum == 7.0
