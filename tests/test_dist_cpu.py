"""Multi-process path on the CPU (gloo, world_size 2): the allgather adapter that shards R1CSProof::prove
across ranks (spg.torch_allgather -> spg_set_comm) carries each rank's partial round sums to every rank,
and the C-side combine (hostcheck's copy of Prover::sum_ranks) adds them exactly mod q."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import spg

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hc = ctypes.CDLL(os.path.join(ROOT, "spartan-parallel_amd", "lib", "libspg_hostcheck.so"))
        fn = spg.torch_allgather(dist)
        rng = np.random.default_rng(100 + rank)
        mine = rng.integers(0, 2**63, (3, 4), dtype=np.uint64)
        mine[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
        out = np.zeros((3, 4), dtype=np.uint64)
        rc = hc.spgh_allgather_sum(fn, None, world, mine.ctypes.data_as(ctypes.c_void_p),
                                   out.ctypes.data_as(ctypes.c_void_p))
        # raw gather through the same adapter: rank-ordered concatenation
        raw = (ctypes.c_uint8 * (8 * world))()
        send = (ctypes.c_uint8 * 8)(*([rank + 1] * 8))
        rc2 = fn(None, ctypes.addressof(send), 8, ctypes.addressof(raw))
        q.put((rank, rc, rc2, mine.tolist(), out.tolist(), list(raw)))
    finally:
        dist.destroy_process_group()


def test_allgather_sum_two_ranks(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    res.sort()
    parts = [np.array(r[3], dtype=np.uint64) for r in res]
    expect = oracle.fq_op("add", parts[0], parts[1])
    for rank, rc, rc2, _, out, raw in res:
        assert rc == 0 and rc2 == 0
        assert np.array_equal(np.array(out, dtype=np.uint64), expect)
        assert raw == [1] * 8 + [2] * 8


def _msm_worker(rank, world, port, q):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import pyoracle
    import shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 37  # ragged split over the ranks
        pts = pyoracle.gens_stream(b"spg_bench_msm", n + 1)[:n]
        rng = np.random.default_rng(7)
        Z = pyoracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * n, dtype=np.uint8).tobytes())
        got, _ = shard.sharded_msm(dist, lambda lo, hi: pyoracle.msm_partial(pts[lo:hi], Z[lo:hi]), n)
        q.put((rank, got, pyoracle.msm(pts, Z)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_msm_matches_single(oracle, world):
    """contiguous shards, one allgather of uncompressed partials, exact host sum == the
    unsharded MSM (partials from the CPU oracle; tests/test_gpu_dist.py runs the device partials)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_msm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, got, ref in res:
        assert got == ref, rank


def test_shard_chunks_cover():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))
    import shard

    for n in (0, 1, 7, 64, 65537):
        for w in (1, 2, 3, 8):
            cs = [shard.chunk(n, r, w) for r in range(w)]
            assert cs[0][0] == 0 and cs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(cs, cs[1:]))
            assert max(h - l for l, h in cs) - min(h - l for l, h in cs) <= 1
