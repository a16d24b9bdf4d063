"""Time-sharded smoothing: one long video split along time over ranks.

SURVEY.md §8(e): the batch of trajectories normally shards with no exchange
(``eks_amd.dist``).  When there are too few trajectories to fill the GPUs
(configs 2, 3 and 5: 1-8 videos of 50k frames), the time axis is split
instead: rank k holds frames [t_base_k, t_base_k + T_k) of every trajectory,
runs the chunked scan of eks_smooth on its own frames, and the ranks exchange
two small per-trajectory aggregates (the segment's filtering element, then its
smoothing map: ~100 doubles per trajectory) with ``all_gather``.  The
reference has no such path (its smoother is one sequential loop,
eks/ensemble_kalman.py:59-164); the results equal ``batch.smooth``'s to rounding.

    phase 1  K1 + segment element        -> all_gather -> combine(kind 0)
    phase 2  K2 + K3 (from the state)    -> all_gather -> combine(kind 1)
    phase 3  K4 + K5 (from the mean)     -> out, nll share (all_reduce sum)

``smooth_segments`` runs every segment in one process (one GPU) with the same
kernels, which is how the single-GPU tests check the exchange algebra.
"""
from __future__ import annotations

from . import _lib, batch


def elem_len(r: int) -> int:
    """Doubles per filtering element (A, b, C, eta, J; C and J packed)."""
    return r * r + 2 * r + r * (r + 1)


def map_len(r: int) -> int:
    return r * r + r


def state_len(r: int) -> int:
    return r + r * (r + 1) // 2


class Segment:
    """The frames [t_base, t_base + T) of B trajectories, T_total frames long.

    Holds the workspace that must survive phases 1..3 and issues the three
    eks_smooth_seg phases on the current stream."""

    def __init__(self, obs, params, *, n: int, r: int, t_base: int, T_total: int,
                 mode: str = "median", flags: int = 0, out=None, slot: str = "seg0",
                 want_out: bool = True, want_ms: bool = False):
        torch = _lib.require_gpu()
        if isinstance(obs, batch.Yev):
            B, T, E, nn = obs.shape
            self.dt, self.ptr, self.strides = obs.code, obs.buf.data_ptr(), (0, 0, 0, 0)
            if mode != obs.mode:
                raise ValueError("the hand-off planes were made in another averaging mode")
        else:
            if obs.dim() != 4:
                raise ValueError("obs must be viewed as (B, T, E, n)")
            B, T, E, nn = obs.shape
            if obs.dtype not in (torch.float32, torch.float64):
                raise TypeError("obs must be float32 or float64")
            self.dt = _lib.EKS_F32 if obs.dtype == torch.float32 else _lib.EKS_F64
            self.ptr, self.strides = obs.data_ptr(), obs.stride()
        if nn != n:
            raise ValueError(f"obs has {nn} coordinates, expected n={n}")
        if mode not in ("median", "mean"):
            raise ValueError(f"{mode} averaging not supported")
        if params.shape != (B, batch.param_len(n, r)) or params.dtype != torch.float64 \
                or not params.is_contiguous():
            raise ValueError(f"params must be a contiguous ({B}, {batch.param_len(n, r)}) "
                             "float64 tensor")
        if not 0 <= t_base <= T_total - T:
            raise ValueError(f"frames [{t_base}, {t_base + T}) outside [0, {T_total})")
        dev = params.device
        self.obs, self.params = obs, params  # keep the buffers alive across phases
        self.B, self.T, self.E, self.n, self.r = B, T, E, n, r
        self.t_base, self.T_total, self.flags = t_base, T_total, flags
        self.mode = _lib.EKS_MEDIAN if mode == "median" else _lib.EKS_MEAN
        if want_out and out is None:
            out = torch.empty((T, B, n), dtype=torch.float64, device=dev).permute(1, 0, 2)
        self.out = out if want_out else None  # None: filter only (NLL), phases 1-2
        self.ms = (torch.empty((B, T, r), dtype=torch.float64, device=dev)
                   if want_ms and want_out else None)
        self.nll = torch.empty((B,), dtype=torch.float64, device=dev)
        self.status = torch.empty((B,), dtype=torch.int32, device=dev)
        lib = _lib.load()
        self.ws = batch.workspace(lib.eks_smooth_seg_workspace_bytes(B, T, n, r), dev, slot=slot)
        self.elem = torch.empty((B, elem_len(r)), dtype=torch.float64, device=dev)
        self.map = torch.empty((B, map_len(r)), dtype=torch.float64, device=dev)
        self.state = torch.empty((B, state_len(r)), dtype=torch.float64, device=dev)
        self.mean = torch.empty((B, r), dtype=torch.float64, device=dev)

    @property
    def first(self) -> bool:
        return self.t_base == 0

    @property
    def last(self) -> bool:
        return self.t_base + self.T == self.T_total

    def phase(self, k: int, seg_in=None, stream=None) -> None:
        seg_out = {1: self.elem, 2: self.map if self.out is not None else None, 3: None}[k]
        ob, ot, oj = self.out.stride() if self.out is not None else (0, 0, 0)
        sb, st, se, sj = self.strides
        _lib.check(_lib.load().eks_smooth_seg(
            self.ptr, self.dt, self.B, self.T, self.E, self.n, self.r, sb, st, se, sj,
            self.mode, self.params.data_ptr(),
            self.out.data_ptr() if self.out is not None else None, ob, ot, oj,
            self.ms.data_ptr() if self.ms is not None else None, self.nll.data_ptr(), self.ws.data_ptr(), self.ws.numel(), self.flags,
            self.status.data_ptr(), self.t_base, self.T_total, k,
            seg_in.data_ptr() if seg_in is not None else None,
            seg_out.data_ptr() if seg_out is not None else None, _lib.stream_ptr(stream)),
            f"eks_smooth_seg(phase {k})")


def combine(kind: int, gathered, nseg: int, self_idx: int, r: int, out, status=None,
            stream=None) -> None:
    """eks_seg_combine on (nseg, B, ·) gathered aggregates -> out (B, ·)."""
    B = out.shape[0]
    if gathered.shape[0] != nseg or gathered.shape[1] != B or not gathered.is_contiguous():
        raise ValueError("gathered aggregates must be a contiguous (nseg, B, ·) tensor")
    _lib.check(_lib.load().eks_seg_combine(
        kind, B, nseg, self_idx, r, gathered.data_ptr(), out.data_ptr(),
        status.data_ptr() if status is not None else None, _lib.stream_ptr(stream)),
        "eks_seg_combine")


def split_frames(T_total: int, nseg: int, k: int) -> tuple[int, int]:
    """(t_base, T) of segment k when T_total frames are split as evenly as
    possible into nseg contiguous segments."""
    if not 0 <= k < nseg or nseg > T_total:
        raise ValueError(f"cannot give segment {k} of {nseg} from {T_total} frames")
    q, rem = divmod(T_total, nseg)
    t0 = k * q + min(k, rem)
    return t0, q + (1 if k < rem else 0)


def smooth_segments(obs, params, *, n: int, r: int, nseg: int, mode: str = "median",
                    flags: int = 0, out=None, want_out: bool = True, want_ms: bool = False):
    """All nseg segments of the time-sharded path in one process (one GPU):
    the same three phases and two combines, with torch.stack standing in for
    the all_gather.  Returns dict(out (B, T, n) or None, ms (B, T, r) or None,
    nll (B,), status (B,)); want_out=False is the filter-only NLL (phases 1-2)."""
    torch = _lib.require_gpu()
    B, T = obs.shape[0], obs.shape[1]
    if not want_out:
        out = None
    elif out is None:
        out = torch.empty((T, B, n), dtype=torch.float64, device=obs.device).permute(1, 0, 2)
    segs = []
    for k in range(nseg):
        t0, tk = split_frames(T, nseg, k)
        segs.append(Segment(obs[:, t0:t0 + tk], params, n=n, r=r, t_base=t0, T_total=T,
                            mode=mode, flags=flags, slot=f"seg{k}", want_out=want_out,
                            want_ms=want_ms,
                            out=out[:, t0:t0 + tk] if want_out else None))
    for s in segs:
        s.phase(1)
    elems = torch.stack([s.elem for s in segs])
    for k, s in enumerate(segs):
        if k:
            combine(0, elems, nseg, k, r, s.state, s.status)
        s.phase(2, s.state if k else None)
    if want_out:
        _backward(segs, r)
    status = segs[0].status.clone()
    for s in segs[1:]:
        status |= s.status
    ms = torch.cat([s.ms for s in segs], dim=1) if want_ms and want_out else None
    return dict(out=out, ms=ms, nll=sum(s.nll for s in segs), status=status)


def _backward(segs, r):
    import torch
    nseg = len(segs)
    maps = torch.stack([s.map for s in segs])
    for k, s in enumerate(segs):
        if k < nseg - 1:
            combine(1, maps, nseg, k, r, s.mean, s.status)
        s.phase(3, s.mean if k < nseg - 1 else None)


def _all_gather(x, group):
    """all_gather of a (B, ·) CUDA tensor into (world, B, ·).  RCCL gathers in
    HBM; gloo (the CPU test backend) goes through a host copy."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x.unsqueeze(0).contiguous()
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        g = torch.empty((world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(g, x.contiguous(), group=group)
        return g
    parts = [torch.empty(x.shape, dtype=x.dtype) for _ in range(world)]
    dist.all_gather(parts, x.cpu(), group=group)
    return torch.stack(parts).to(x.device)


def smooth_time_sharded(obs, params, *, n: int, r: int, t_base: int, T_total: int,
                        mode: str = "median", flags: int = 0, group=None, out=None,
                        want_nll: bool = False, want_out: bool = True,
                        want_ms: bool = False):
    """This rank's segment of a time-sharded smooth: obs (B, T, E, n) holds
    frames [t_base, t_base + T) of every trajectory; segments are ordered by
    rank (rank k holds segment k) and together cover [0, T_total).

    Returns dict(out (B, T, n) and ms (B, T, r) (if want_ms) of this
    segment, status (B,) this segment's
    flags, nll (B,) summed over all segments if want_nll); want_out=False is
    the filter-only NLL (phases 1-2, one exchange + the NLL sum)."""
    import torch.distributed as dist
    single = not dist.is_initialized()  # one process: a single segment, no exchange
    world = 1 if single else dist.get_world_size(group)
    rank = 0 if single else dist.get_rank(group)
    seg = Segment(obs, params, n=n, r=r, t_base=t_base, T_total=T_total, mode=mode,
                  flags=flags, out=out, slot="seg", want_out=want_out, want_ms=want_ms)
    if (rank == 0) != seg.first or (rank == world - 1) != seg.last:
        raise ValueError(f"rank {rank} of {world} holds frames [{t_base}, {t_base + seg.T}) "
                         f"of {T_total}: segments must be ordered by rank")
    seg.phase(1)
    elems = _all_gather(seg.elem, group)
    if rank:
        combine(0, elems, world, rank, r, seg.state, seg.status)
    seg.phase(2, seg.state if rank else None)
    if want_out:
        maps = _all_gather(seg.map, group)
        if rank < world - 1:
            combine(1, maps, world, rank, r, seg.mean, seg.status)
        seg.phase(3, seg.mean if rank < world - 1 else None)
    nll = None
    if want_nll or not want_out:
        nll = _all_gather(seg.nll[:, None], group).sum(0)[:, 0]
    return dict(out=seg.out, ms=seg.ms, status=seg.status, nll=nll)
