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
