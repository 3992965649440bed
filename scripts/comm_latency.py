"""Per-exchange latency of libspg's two SPMD transports: the callback transport over
torch.distributed gloo with 2 processes on this box, and the native RCCL transport on one rank (RCCL rejects two
ranks on one GPU, so a 2-rank RCCL figure needs a 2-GPU node). 104-byte payloads: a layer round's status word +
(e0, e2, e3). Prints one JSON line."""
import json
import os
import socket
import sys
import time

import torch.multiprocessing as mp

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
N = 300


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPG_PIN="0")
    import torch
    import torch.distributed as dist

    import spg

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = spg.Context(0)
    ctx.set_comm(rank, world, spg.torch_allgather(dist))
    msg = bytes(104)
    for _ in range(20):
        ctx.comm_allgather(msg, world)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(N):
        ctx.comm_allgather(msg, world)
    cb_us = (time.perf_counter() - t0) / N * 1e6
    src = torch.zeros(104, dtype=torch.uint8)
    outs = [torch.empty_like(src) for _ in range(world)]
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(N):
        dist.all_gather(outs, src)
    raw_us = (time.perf_counter() - t0) / N * 1e6
    q.put((rank, cb_us, raw_us))
    dist.destroy_process_group()


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)])
    for p in ps:
        p.join(timeout=60)
    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd")]
    import spg

    c = spg.Context(0)
    c.set_comm_rccl(0, 1)
    msg = bytes(104)
    for _ in range(20):
        c.comm_allgather(msg, 1)
    t0 = time.perf_counter()
    for _ in range(N):
        c.comm_allgather(msg, 1)
    rccl_us = (time.perf_counter() - t0) / N * 1e6
    print(json.dumps({"payload_bytes": 104, "callback_gloo_2ranks_us": round(max(r[1] for r in res), 1),
                      "torch_gloo_all_gather_2ranks_us": round(max(r[2] for r in res), 1),
                      "rccl_native_1rank_us": round(rccl_us, 1)}))


if __name__ == "__main__":
    main()
