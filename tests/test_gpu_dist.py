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
    # one shared matrix, instances of different widths: rank 1's first instance (2) is narrower than the matrix
    # (instance 0's width), so its fused phase-2 fold could not write the ABC ping-pong buffer
    "p4_shared_mixed_inputs": ([64] * 4, [8, 8, 4, 8], 2, True, [128, 128, 64, 128]),
}


def _wl(case, **kw):
    import workload

    nc, npf, nws, shared, *rest = CASES[case]
    return workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared,
                                 num_inputs=rest[0] if rest else None, **kw)
WORLD = {"p5_uneven": 4}  # ceil split would leave rank 3 empty; the balanced split gives 2,1,1,1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q, bad_shard=False, failpoint=None, cb_fail=False):
    import sys

    if failpoint:  # read by libspg at its first check (tests only): the last rank fails inside a phase-1 round
        os.environ["SPG_FAILPOINT"] = failpoint
        os.environ["SPG_FAILPOINT_RANK"] = str(world - 1)
    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import spg
    import workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SPG_PIN"] = "0"  # several ranks share the test box's GPU (and would pick the same CPU domain)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = _wl(case)
        ctx = spg.Context(0)
        ctx.set_comm(rank, world, spg.torch_allgather(dist))
        gens = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
        v = workload.CViews(wl)
        inst = spg.R1CSInst(ctx, v.inst)
        shard = spg.shard_range(wl.P, rank, world)
        if bad_shard and rank == world - 1:
            shard = (0, 1)  # this rank uploads a shard that does not hold its instances
        wit = spg.R1CSWitness(ctx, v.secs, wl.nws, shard=shard)
        tr = _caller_transcript(b"r1cs_test", rank == world - 1) if cb_fail else spg.Transcript(b"r1cs_test")
        pf, ch = spg.r1cs_prove(ctx, gens, inst, wit, wl.P, wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs,
                                wl.num_inputs, tr, spg.RandomTape(b"proof", workload.tape_seed()))
        q.put((rank, pf, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _caller_transcript(label, refuse):
    """the caller's own merlin transcript (the oracle's restatement) behind spg_transcript_new_callbacks; with
    `refuse` its 40th append raises, i.e. the callback fails mid-proof on this rank only"""
    import pyoracle
    import spg

    t = pyoracle.OracleTranscript(label)
    n = [0]

    def app(lbl, msg):
        n[0] += 1
        if refuse and n[0] == 40:
            raise RuntimeError("caller transcript refused")
        t.append_message(lbl, msg)

    return spg.Transcript.from_callbacks(app, t.challenge_bytes)


def _collect(ps, q, world, timeout):
    """every rank's result, or a failure naming the ranks that never reported (blocked in an exchange)"""
    import queue

    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=timeout))
    except queue.Empty:
        pass
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.terminate()
    assert len(res) == world, f"only ranks {sorted(r[0] for r in res)} of {world} returned: a rank is blocked"
    return sorted(res, key=lambda r: r[0])


def _run(case, world, bad_shard=False, failpoint=None, cb_fail=False, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, case, q, bad_shard, failpoint, cb_fail))
          for r in range(world)]
    for p in ps:
        p.start()
    return _collect(ps, q, world, timeout)


@pytest.mark.parametrize("case", sorted(CASES))
def test_sharded_proof_matches_oracle(oracle, case):
    import workload

    wl = _wl(case)
    ref, _ = oracle.r1cs_prove(wl, workload.tape_seed())
    for rank, pf, err in _run(case, WORLD.get(case, 2)):
        assert err is None, err
        assert pf == ref, f"rank {rank} proof differs"


def test_sharded_bad_shard_fails_every_rank():
    res = _run("p3_uneven", 2, bad_shard=True)
    assert all(pf is None and err for _, pf, err in res), res


def test_sharded_r1cs_rank_failure_fails_every_rank():
    """a failure on one rank inside a phase-1 round of a sharded R1CSProof (test failpoint, before that round's
    exchange): the failing rank takes part in the next exchange of the plan with its status, so every rank returns an
    error and none blocks in a later exchange"""
    res = _run("p4_ragged_3secs", 2, failpoint="r1cs_round", timeout=120)
    for rank, pf, err in res:
        assert pf is None and err, f"rank {rank} did not fail: {res}"
    assert "failpoint" in res[1][2] and "peer rank failed" in res[0][2], res


def test_sharded_r1cs_callback_failure_fails_every_rank():
    """the caller transcript of one rank fails mid-proof: its failure rides the next exchange as that rank's status
    (TrFailScope), so the healthy rank returns an error too instead of a proof built on zeroed challenges"""
    res = _run("p4_ragged_3secs", 2, cb_fail=True, timeout=120)
    for rank, pf, err in res:
        assert pf is None and err, f"rank {rank} did not fail: {res}"
    assert "SPG_E_CALLBACK" in res[1][2], res


# ---- sharded SPARK (SparseMatPolyEvalProof over W processes; multi_evaluate rows split) ----------
SPARK_SHARD_CASES = {  # (R1CS shape as in r1cs_cases, world sizes)
    "p2_x64_2secs": [2, 4, 3],
    "p2_x256": [2, 4],
    "p1_x16": [8],
}


def _spark_worker(rank, world, port, case, q, failpoint=None, cb_fail=False, rccl=False):
    import sys

    if failpoint:  # read by libspg at its first check (tests only): this rank fails inside a sharded layer
        os.environ["SPG_FAILPOINT"] = failpoint
        os.environ["SPG_FAILPOINT_RANK"] = str(world - 1)

    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
    import torch.distributed as dist

    import numpy as np

    import spg
    import workload
    from r1cs_cases import GPU_SPARK_CASES, SPARK_CASES

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SPG_PIN"] = "0"  # several ranks share the test box's GPU (and would pick the same CPU domain)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cases = dict(SPARK_CASES, **GPU_SPARK_CASES)
        nc, npf, nws, shared = cases[case]
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, shared_instance=shared)
        nx = (wl.max_num_cons - 1).bit_length()
        ny = (wl.num_vars - 1).bit_length()
        rx, ry = _spark_point(nx, ny)
        if rccl:  # one GPU per rank, libspg's own transport
            ctx = spg.Context(rank)
            ctx.set_comm_rccl(rank, world, dist)
        else:
            ctx = spg.Context(0)
            ctx.set_comm(rank, world, spg.torch_allgather(dist))
        v = workload.CViews(wl)
        gens_nnz = len(wl.entries) * max(max(int(m.shape[0]) for m in mats) for mats in wl.entries)
        comm = spg.SparkCommitment(ctx, v.inst, b"gens_r1cs_eval", gens_nnz, 3)
        inst = spg.R1CSInst(ctx, v.inst)
        evals = spg.r1cs_multi_evaluate(ctx, inst, len(wl.entries), rx, ry)
        tr = _caller_transcript(b"spark_test", rank == world - 1) if cb_fail else spg.Transcript(b"spark_test")
        proof = comm.prove(rx, ry, evals, tr, spg.RandomTape(b"proof", workload.tape_seed()))
        q.put((rank, comm.bytes, np.asarray(evals).tobytes(), proof, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _spark_point(nx, ny):
    import numpy as np

    import pyoracle

    rng = np.random.default_rng(3)
    r = pyoracle.fq_from_bytes_wide(rng.integers(0, 256, 64 * (nx + ny), dtype=np.uint8).tobytes())
    return r[:nx], r[nx:]


@pytest.mark.parametrize("case,world", [(c, w) for c, ws in sorted(SPARK_SHARD_CASES.items()) for w in ws])
def test_sharded_spark_matches_oracle(oracle, case, world):
    """every rank of a W-process SPARK proof emits the single-process oracle's commitment, evaluations and proof"""
    import numpy as np

    import workload
    from test_oracle_spark import spark_inputs

    wl, rx, ry = spark_inputs(oracle, case)
    rcomm, ref, ok = oracle.spark_prove(wl, rx, ry, workload.tape_seed())
    assert ok
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_spark_worker, args=(r, world, port, case, qq)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([qq.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    evs = {r[2] for r in res}
    assert len(evs) == 1, "ranks disagree on multi_evaluate"
    for rank, cm, _, pf, err in res:
        assert err is None, err
        assert cm == rcomm, f"rank {rank} commitment differs"
        assert pf == ref, f"rank {rank} proof differs"


def test_sharded_spark_callback_failure_fails_every_rank():
    """one rank's caller transcript fails mid-proof of a sharded SPARK proof: every rank returns an error"""
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_spark_worker, args=(r, world, port, "p2_x64_2secs", qq, None, True))
          for r in range(world)]
    for p in ps:
        p.start()
    res = _collect(ps, qq, world, 120)
    for rank, _, _, pf, err in res:
        assert pf is None and err, f"rank {rank} did not fail: {res}"


def test_sharded_spark_rank_failure_fails_every_rank():
    """a failure on one rank inside a sharded SPARK layer (test failpoint) reaches every rank through the next
    exchange (skip mode): all ranks return an error, none blocks in a collective"""
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_spark_worker, args=(r, world, port, "p2_x64_2secs", qq, "spark_layer"))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([qq.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for rank, _, _, pf, err in res:
        assert pf is None and err, f"rank {rank} did not fail: {res}"


# ---- libspg's own RCCL transport (spg_set_comm_rccl) ----------------------------------------------------------
def test_rccl_transport_one_rank(ctx):
    """the RCCL transport on one rank: the communicator initialises on the context's device, an allgather moves the
    bytes through ncclAllGather on the context stream, and a proof still runs with it installed (one rank never
    exchanges). Two ranks need two GPUs (RCCL rejects two ranks on one device): test_rccl_two_gpus below."""
    import time

    import spg

    c = spg.Context(0)
    c.set_comm_rccl(0, 1)
    for n in (1, 8, 104, 4096):
        data = bytes((i * 7 + n) % 256 for i in range(n))
        assert c.comm_allgather(data, 1) == [data]
    t0 = time.perf_counter()
    for _ in range(200):
        c.comm_allgather(b"x" * 104, 1)
    us = (time.perf_counter() - t0) / 200 * 1e6
    print(f"RCCL 1-rank exchange of 104 bytes: {us:.1f} us")
    c.close()


def _rccl_worker(rank, world, port, case, q):
    import sys

    sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd")]
    import torch.distributed as dist

    import spg
    import workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = _wl(case)
        ctx = spg.Context(rank)
        ctx.set_comm_rccl(rank, world, dist)
        gens = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
        v = workload.CViews(wl)
        inst = spg.R1CSInst(ctx, v.inst)
        wit = spg.R1CSWitness(ctx, v.secs, wl.nws, shard=spg.shard_range(wl.P, rank, world))
        pf, _ = spg.r1cs_prove(ctx, gens, inst, wit, wl.P, wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs,
                               wl.num_inputs, spg.Transcript(b"r1cs_test"), spg.RandomTape(b"proof", workload.tape_seed()))
        q.put((rank, pf, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_two_gpus_sharded_r1cs(oracle):
    """a sharded R1CSProof over the RCCL transport, one process per GPU (needs >= 2 GPUs on the box)"""
    import torch

    import workload

    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one GPU per rank; this box has one")
    case = "p4_ragged_3secs"
    ref, _ = oracle.r1cs_prove(_wl(case), workload.tape_seed())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rccl_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for rank, pf, err in res:
        assert err is None, err
        assert pf == ref, f"rank {rank} proof differs"


def test_rccl_two_gpus_sharded_spark(oracle):
    """a sharded SPARK proof over the RCCL transport, one process per GPU (needs >= 2 GPUs on the box): every rank
    emits the single-process oracle's commitment and proof"""
    import torch

    import workload
    from test_oracle_spark import spark_inputs

    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one GPU per rank; this box has one")
    case = "p2_x64_2secs"
    wl, rx, ry = spark_inputs(oracle, case)
    rcomm, ref, ok = oracle.spark_prove(wl, rx, ry, workload.tape_seed())
    assert ok
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_spark_worker, args=(r, 2, port, case, qq, None, False, True)) for r in range(2)]
    for p in ps:
        p.start()
    res = _collect(ps, qq, 2, 300)
    for rank, cm, _, pf, err in res:
        assert err is None, err
        assert cm == rcomm and pf == ref, f"rank {rank} differs"
