"""One MSM split over ranks (SURVEY.md 8e "Single large MSM (config 2)"): contiguous chunks of the
(scalar, generator) pairs per rank, one uncompressed partial sum per rank (spg_msm_partial), one allgather of
the 128-byte partials (RCCL over xGMI on GPUs, gloo in the CPU tests), an exact group addition of the partials
and the encoding on the host (spg_points_sum_compress). The result is the compressed point
GroupElement::vartime_multiscalar_mul (src/group.rs:98-116) returns for the whole MSM."""
import numpy as np

import spg


def chunk(n, rank, world):
    """[lo, hi) of rank's contiguous share of n pairs (the first n % world ranks take one more)"""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def allgather_bytes(dist, data, device=None):
    """rank-ordered list of every rank's `data` (same length on all ranks)"""
    import torch

    t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [bytes(o.cpu().numpy().tobytes()) for o in out]


def sharded_msm(dist, partial, n, device=None):
    """partial(lo, hi) -> 128-byte partial sum of pairs [lo, hi); returns (32-byte compressed sum, my partial)"""
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = chunk(n, rank, world)
    mine = partial(lo, hi)
    assert len(mine) == 128
    parts = allgather_bytes(dist, mine, device)
    return spg.points_sum_compress(parts), mine


def gpu_partial(gens, scalars):
    """partial(lo, hi) over a device generator set and host scalars (Montgomery limbs, n x 4 u64)"""
    s = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)

    def f(lo, hi):
        return gens.msm_partial(s[lo:hi], gen_offset=lo)

    return f


def gpu_partial_resident(gens, buf):
    """partial(lo, hi) over a device generator set and device-resident scalars (a spg.Buf uploaded once)"""

    def f(lo, hi):
        return gens.msm_partial_buf(buf, offset=lo, n=hi - lo, gen_offset=lo)

    return f
