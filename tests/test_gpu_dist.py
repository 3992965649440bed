"""Sharded R1CSProof::prove: two to four processes share the one GPU of the test box (gloo for the per-round
allgather), each holding a balanced share of the instances (spg_set_comm + spg_r1cs_witness_new_shard).
Every rank must emit exactly the proof bytes of the single-process CPU oracle; a rank whose witness shard
does not match its instance range makes every rank fail (no rank blocks in an allgather)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {
    "p2_x64": ([64, 64], [16, 16], 1, False),
    "p4_ragged_3secs": ([32, 16, 8, 4], [8, 4, 2, 1], 3, False),
    "p4_shared": ([64] * 4, [8, 8, 4, 8], 2, True),
    "p3_uneven": ([16, 16, 16], [4, 4, 4], 1, False),
    "p5_uneven": ([16, 32, 16, 8, 16], [4, 2, 4, 4, 2], 2, False),
}
WORLD = {"p5_uneven": 4}  # ceil split would leave rank 3 empty; the balanced split gives 2,1,1,1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q, bad_shard=False):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd")]
    import torch.distributed as dist

    import spg
    import workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nc, npf, nws, shared = CASES[case]
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
        ctx = spg.Context(0)
        ctx.set_comm(rank, world, spg.torch_allgather(dist))
        gens = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
        v = workload.CViews(wl)
        inst = spg.R1CSInst(ctx, v.inst)
        shard = spg.shard_range(wl.P, rank, world)
        if bad_shard and rank == world - 1:
            shard = (0, 1)  # this rank uploads a shard that does not hold its instances
        wit = spg.R1CSWitness(ctx, v.secs, wl.nws, shard=shard)
        pf, ch = spg.r1cs_prove(ctx, gens, inst, wit, wl.P, wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs,
                                wl.num_inputs, spg.Transcript(b"r1cs_test"), spg.RandomTape(b"proof", workload.tape_seed()))
        q.put((rank, pf, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(case, world, bad_shard=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, case, q, bad_shard)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("case", sorted(CASES))
def test_sharded_proof_matches_oracle(oracle, case):
    import workload

    nc, npf, nws, shared = CASES[case]
    wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
    ref, _ = oracle.r1cs_prove(wl, workload.tape_seed())
    for rank, pf, err in _run(case, WORLD.get(case, 2)):
        assert err is None, err
        assert pf == ref, f"rank {rank} proof differs"


def test_sharded_bad_shard_fails_every_rank():
    res = _run("p3_uneven", 2, bad_shard=True)
    assert all(pf is None and err for _, pf, err in res), res
