#!/usr/bin/env python3
"""Benchmark for the MI355X Spartan prover (libspg.so), one JSON line on rank 0.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 launched under
torch.distributed.run, one rank per GPU.

--workload snark (default, the headline metric): SNARK::prove (src/lib.rs:971-2746)
    on a synthetic 2^20-constraint program (2 block types x 2^9 executions x 2^10 constraints), instances
    encoded and witness resident in HBM before the timed region; every step produces the full bincode(SNARK),
    compared byte-for-byte with the CPU oracle's. Multi-GPU: independent replicas (weak scaling).
--workload r1cs: the block R1CSProof::prove alone (src/r1csproof.rs:210-685); --mode shard splits ONE proof
    over the ranks by instance with a per-round allgather (spg_set_comm).
--workload spark: SURVEY 8d config 5, multi_evaluate + SparseMatPolyEvalProof::prove at 3 x 2^k nonzeros.
--workload msm: SURVEY 8d config 2, one 2^16-point MSM split over the ranks (spg_msm_partial + allgather +
    spg_points_sum_compress, strong scaling).

`roofline` is computed for the kernel with the largest device time among those with an algorithmic byte
model (libspg's per-launch HIP-event timing on its context stream, spg_prof_read, taken in a separate pass
after the timed steps); `traffic` comes from the committed PMC summary (profiles/r02_pmc_traffic.json).
`cpu_baseline` is the C++ CPU restatement of the reference (oracle/, 1 thread) on rank 0 at N = 1.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (/opt/skills/guides/MI355X_MICROARCH.md)
GENS_LABEL = b"gens_r1cs_sat"
GENS_NUM_VARS = 1 << 24  # TOTAL_NUM_VARS_BOUND = 10^7 -> 2^24 (examples/interface.rs:557-563)
CONFIGS = {
    # name: (num_cons per instance, num_proofs per instance, witness sections)
    "r1cs_2e20": ([1024, 1024], [512, 512], 1),
    "r1cs_2e16": ([1024, 1024], [32, 32], 1),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="r1cs_2e20", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default=None, choices=["replicas", "shard"],
                    help="N > 1: replicas (independent proofs per rank) or shard (one proof split over the ranks); "
                         "default: shard for --workload spark / msm, replicas otherwise")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl with a GPU)")
    ap.add_argument("--log-msm", type=int, default=16, help="msm: 2^k (scalar, generator) pairs")
    ap.add_argument("--workload", default="snark", choices=["snark", "r1cs", "spark", "msm"],
                    help="snark: the headline metric (SNARK::prove, SURVEY 8d config 3); r1cs: its block "
                         "R1CSProof::prove alone; spark: SURVEY 8d config 5 (SPARK)")
    ap.add_argument("--log-cons", type=int, default=10, help="snark: 2^k constraints per block")
    ap.add_argument("--log-proofs", type=int, default=9, help="snark: 2^k executions per block")
    ap.add_argument("--log-nnz", type=int, default=24, help="spark: 2^k nonzeros per matrix (x3 matrices)")
    ap.add_argument("--cpu-log-nnz", type=int, default=15, help="spark: CPU baseline sample size")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r02_pmc_traffic.json"),
                    help="per-launch HBM bytes from rocprofv3 --pmc (scripts/pmc_traffic.py), if present")
    return ap.parse_args()


def main():
    a = parse()
    if a.workload == "spark":
        return main_spark(a)
    if a.workload == "snark":
        return main_snark(a)
    if a.workload == "msm":
        return main_msm(a)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend)
    ndev = torch.cuda.device_count()
    gpu = local % ndev if ndev else local  # ranks share a GPU only when there are fewer GPUs (rehearsals)
    if torch.cuda.is_available():
        torch.cuda.set_device(gpu)

    import spg
    import workload

    nc, npf, nws = CONFIGS[a.config]
    shard = (a.mode or "replicas") == "shard" and world > 1
    ctx = spg.Context(gpu)
    if shard:
        nc, npf = nc * world, npf * world  # one proof over world x the per-GPU instances
        p0, p1 = spg.shard_range(len(nc), rank, world)
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, instances=range(p0, p1))
        dev = f"cuda:{gpu}" if backend == "nccl" else "cpu"
        ctx.set_comm(rank, world, spg.torch_allgather(dist, device=dev))
    else:
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, seed=0x5350415254414E31 + rank)
    seed = workload.tape_seed()
    gens = spg.R1CSGens(ctx, GENS_LABEL, GENS_NUM_VARS)
    views = workload.CViews(wl)
    inst = spg.R1CSInst(ctx, views.inst)

    def upload():
        return spg.R1CSWitness(ctx, views.secs, wl.nws, shard=(p0, p1) if shard else None)

    wit = upload()

    def step():
        t = spg.Transcript(b"r1cs_bench")
        tape = spg.RandomTape(b"proof", seed)
        return spg.r1cs_prove(ctx, gens, inst, wit, wl.P, wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs,
                              wl.num_inputs, t, tape)

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    proofs = set()
    for _ in range(a.steps):
        pf, ch = step()
        proofs.add(hashlib.sha256(pf).hexdigest())
    sync()
    dt = time.perf_counter() - t0
    prof = profile_pass(ctx, step, a.steps)
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    assert len(proofs) == 1, "proof bytes changed between steps"

    # PCIe-inclusive variant: witness upload + prove (reported beside value, never as value)
    t1 = time.perf_counter()
    wit = upload()
    step()
    t_incl = time.perf_counter() - t1

    N = wl.total_constraints // world if shard else wl.total_constraints  # per GPU
    value = N * world * a.steps / dt
    ms = dt / a.steps * 1e3

    # roofline of the dominant modelled kernel (per-launch average, HIP events on the context stream)
    modelled = {k: v for k, v in prof.items() if v[2] > 0}
    dom = max(modelled, key=lambda k: modelled[k][1])
    launches, us, nbytes = modelled[dom]
    achieved = (nbytes / launches) / (us / launches * 1e-6) / 1e9
    traffic = None
    if os.path.exists(a.traffic):
        tr = json.load(open(a.traffic))
        if dom in tr.get("kernels", {}):
            traffic = tr["kernels"][dom]["hbm_bytes_per_launch"]
    roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": nbytes / launches, "avg_launch_us": us / launches, "launches": launches}
    device_ms = sum(v[1] for v in prof.values()) / a.steps / 1e3
    top = sorted(prof.items(), key=lambda kv: -kv[1][1])[:8]
    kernels = {k: {"launches_per_step": v[0] / a.steps, "ms_per_step": round(v[1] / a.steps / 1e3, 3),
                   "GBps": round(v[2] / (v[1] * 1e-6) / 1e9, 1) if v[2] else None} for k, v in top}

    cpu = None
    bitexact = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle  # the checker / CPU baseline only

        pyoracle.build()
        tc = time.perf_counter()
        ref, _ = pyoracle.r1cs_prove(wl, seed, gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS,
                                     label=b"r1cs_bench")
        tcpu = time.perf_counter() - tc
        cpu = {"value": round(N / tcpu, 1), "unit": "constraints/s", "cores": 1, "kind": "port",
               "sample": f"full workload ({N} constraints), one R1CSProof::prove incl. R1CSGens derivation, "
                         f"{tcpu:.2f} s on 1 host thread"}
        bitexact = hashlib.sha256(ref).hexdigest() in proofs

    if rank == 0:
        out = {
            "metric": "R1CS constraints/sec (SNARK::prove) at 2^20 vars; proof bytes bit-exact",
            "value": round(value, 1), "unit": "constraints/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fq252 (8x u32 Montgomery limbs), ristretto255",
            "data": "synthetic (chain-of-squarings R1CS, seeded), random-tape seed fixed",
            "config": {"workload": "R1CSProof::prove, block-sat proof of SNARK::prove (src/r1csproof.rs:210-685)",
                       "num_instances": wl.P, "num_cons": nc, "num_proofs": npf, "witness_sections": nws,
                       "constraints_per_gpu": N, "max_num_inputs": wl.max_num_inputs,
                       "gens": "R1CSGens(gens_r1cs_sat, 2^24)",
                       "parallelism": f"instance-sharded single proof x{world} ({backend})" if shard
                       else f"replicas x{world}"},
            "roofline": roof, "cpu_baseline": cpu, "proof_bitexact_vs_cpu": bitexact,
            "proof_sha256": sorted(proofs)[0][:16], "device_busy_ms_per_step": round(device_ms, 3),
            "value_incl_witness_upload": round(N * world / t_incl, 1), "kernels": kernels,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def profile_pass(ctx, step, steps):
    """per-kernel HIP-event timing (libspg spg_prof_*) of `steps` extra steps run after the timed region, so
    the events never perturb `value`; returns {kernel: (launches, us, algorithmic bytes)} summed over them"""
    ctx.prof_enable(True)
    ctx.prof_read(reset=True)
    for _ in range(steps):
        step()
    prof = ctx.prof_read(reset=True)
    ctx.prof_enable(False)
    return prof


def roofline_of(prof, traffic_file):
    """roofline object for the modelled kernel with the largest device time"""
    modelled = {k: v for k, v in prof.items() if v[2] > 0}
    dom = max(modelled, key=lambda k: modelled[k][1])
    launches, us, nbytes = modelled[dom]
    achieved = (nbytes / launches) / (us / launches * 1e-6) / 1e9
    traffic = None
    if traffic_file and os.path.exists(traffic_file):
        tr = json.load(open(traffic_file))
        if dom in tr.get("kernels", {}):
            traffic = tr["kernels"][dom]["hbm_bytes_per_launch"]
    per = nbytes / launches
    out = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
           "algorithmic_bytes_per_launch": per, "avg_launch_us": us / launches, "launches": launches,
           # a launch that moves < 64 MB cannot approach the HBM peak behind a ~4 us small-launch floor: its
           # regime is the round-trip latency (transcript-sequential rounds over KB-sized vectors), DESIGN.md 4
           "regime": "bandwidth" if per >= (64 << 20) else "latency"}
    return out


def main_snark(a):
    """The headline metric: SNARK::prove (src/lib.rs:971-2746) on the synthetic program of
    workload.SnarkWorkload: 2 block types x 2^log_proofs executions x 2^log_cons constraints (N = 2^20 by
    default), no memory operations, vars_gens = R1CSGens(gens_r1cs_sat, 2^24). A step is one full SNARK::prove
    (witness recurrences, every Hyrax commitment, the block / pairwise / perm-root R1CSProofs with their
    R1CSEvalProofs, perm-product, shift and IO proofs) with the instances encoded (SNARK::encode, preprocessing)
    and block_vars / exec inputs resident in HBM. Multi-GPU: independent replicas (one SNARK per rank)."""
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(a.backend or ("nccl" if torch.cuda.is_available() else "gloo"))
    ndev = torch.cuda.device_count()
    gpu = local % ndev if ndev else local
    if torch.cuda.is_available():
        torch.cuda.set_device(gpu)
    import spg
    import workload

    ctx = spg.Context(gpu)
    t0 = time.perf_counter()
    wl = workload.SnarkWorkload(num_blocks=2, log_cons=a.log_cons, log_proofs=a.log_proofs,
                                num_vars=1 << a.log_cons, seed=0x5350415254414E31 + rank)
    views = workload.SnarkViews(wl)
    t_gen = time.perf_counter() - t0
    seed = workload.tape_seed()
    gens = spg.R1CSGens(ctx, GENS_LABEL, GENS_NUM_VARS)
    t0 = time.perf_counter()
    block = spg.SnarkComp(ctx, views.block, multi=True)
    pairwise = spg.SnarkComp(ctx, views.pairwise)
    perm_root = spg.SnarkComp(ctx, views.perm_root)
    t_encode = time.perf_counter() - t0
    wit = spg.SnarkWitness(ctx, views.inputs)

    def step():
        return spg.snark_prove(ctx, block, pairwise, perm_root, wit, gens, spg.Transcript(b"snark_bench"),
                               spg.RandomTape(b"proof", seed))

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    proofs = set()
    laps = []  # per-prove wall times (a prove returns its bytes, so each step is synchronous)
    for _ in range(a.steps):
        t1 = time.perf_counter()
        proofs.add(hashlib.sha256(step()).hexdigest())
        laps.append(time.perf_counter() - t1)
    sync()
    dt = time.perf_counter() - t0
    prof = profile_pass(ctx, step, a.steps)
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    assert len(proofs) == 1, "proof bytes changed between steps"
    t1 = time.perf_counter()  # PCIe-inclusive variant: witness upload + prove (reported beside value)
    wit = spg.SnarkWitness(ctx, views.inputs)
    proof = step()
    t_incl = time.perf_counter() - t1
    # SNARK::verify of the same proof on the product path (not part of value; reported beside it)
    verify_ok, _ = spg.snark_verify(ctx, block, pairwise, perm_root, views.inputs, gens, spg.Transcript(b"snark_bench"),
                                    proof)
    t1 = time.perf_counter()
    for _ in range(3):
        spg.snark_verify(ctx, block, pairwise, perm_root, views.inputs, gens, spg.Transcript(b"snark_bench"), proof)
    t_verify = (time.perf_counter() - t1) / 3
    N = wl.total_constraints
    value = N * world * a.steps / dt
    top = sorted(prof.items(), key=lambda kv: -kv[1][1])[:10]
    kernels = {n: {"launches_per_step": v[0] / a.steps, "ms_per_step": round(v[1] / a.steps / 1e3, 3),
                   "GBps": round(v[2] / (v[1] * 1e-6) / 1e9, 1) if v[2] else None} for n, v in top}
    cpu, bitexact, cpu_verify_ms = None, None, None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle  # the checker / CPU baseline only

        pyoracle.build()
        ref, rc = pyoracle.snark_prove(wl, seed, gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS,
                                       label=b"snark_bench")
        tcpu = pyoracle.snark_last_prove_us() * 1e-6
        cpu_verify_ms = pyoracle.snark_last_verify_us() * 1e-3
        cpu = {"value": round(N / tcpu, 1), "unit": "constraints/s", "cores": 1, "kind": "port",
               "sample": f"full workload ({N} constraints), one SNARK::prove (instances pre-encoded), "
                         f"{tcpu:.2f} s on 1 host thread; oracle verifier status {rc}"}
        bitexact = hashlib.sha256(ref).hexdigest() in proofs
    if rank == 0:
        print(json.dumps({
            "metric": "R1CS constraints/sec (SNARK::prove) at 2^20 vars; proof bytes bit-exact",
            "value": round(value, 1), "unit": "constraints/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fq252 (8x u32 Montgomery limbs), ristretto255",
            "data": "synthetic program (2 block types, chain-of-squarings blocks, seeded), random-tape seed fixed",
            "config": {"workload": "SNARK::prove (src/lib.rs:971-2746)", "block_types": 2,
                       "constraints_per_block": 1 << a.log_cons, "executions_per_block": 1 << a.log_proofs,
                       "constraints_per_gpu": N, "num_vars": wl.num_vars, "num_ios": wl.num_ios,
                       "gens": "R1CSGens(gens_r1cs_sat, 2^24)", "parallelism": f"replicas x{world}"},
            "roofline": roofline_of(prof, a.traffic), "cpu_baseline": cpu, "proof_bitexact_vs_cpu": bitexact,
            "proof_sha256": sorted(proofs)[0][:16], "proof_bytes": None,
            "device_busy_ms_per_step": round(sum(v[1] for v in prof.values()) / a.steps / 1e3, 3),
            "value_incl_witness_upload": round(N * world / t_incl, 1), "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3),
            "ms_per_step_min": round(min(laps) * 1e3, 3), "verify_ms": round(t_verify * 1e3, 2),
            "verify_ok": verify_ok, "cpu_verify_ms_1thread": None if cpu_verify_ms is None else round(cpu_verify_ms, 1),
            "encode_s": round(t_encode, 3),
            "host_gen_s": round(t_gen, 3), "kernels": kernels}))
    if dist is not None:
        dist.destroy_process_group()


def msm_scalars(n):
    """SURVEY 8d config 2 scalars: uniform Fq (splitmix64 seed 1) with edge cases 0, 1, 2, q-1, q-2, 2^252,
    2^252 - 1, 2^251 in the first 8 slots; Montgomery limbs (n x 4 u64)"""
    import workload

    v, _ = workload.random_fq(n, 1)
    v = [int(x) for x in v]
    Q = workload.Q
    edge = [0, 1, 2, Q - 1, Q - 2, 1 << 252, (1 << 252) - 1, 1 << 251]
    v[: min(8, n)] = edge[: min(8, n)]
    return workload.to_mont_limbs(v)


def main_msm(a):
    """one 2^k-point MSM (GroupElement::vartime_multiscalar_mul, src/group.rs:98-116) against
    MultiCommitGens::new(2^k, b"spg_bench_msm").G, resident in HBM. With N ranks the MSM is split into
    contiguous chunks: each rank computes an uncompressed partial sum (spg_msm_partial), the
    128-byte partials are allgathered over RCCL and added exactly on the host (shard.py) -> strong scaling.
    A step is one whole MSM ending in the 32-byte compressed result on every rank."""
    import torch

    import shard

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend)
    ndev = torch.cuda.device_count()
    gpu = local % ndev if ndev else local
    if torch.cuda.is_available():
        torch.cuda.set_device(gpu)
    import spg

    ctx = spg.Context(gpu)
    n = 1 << a.log_msm
    gens = spg.Gens(ctx, n, b"spg_bench_msm")
    sc = msm_scalars(n)
    partial = shard.gpu_partial(gens, sc)
    dev = f"cuda:{gpu}" if backend == "nccl" else None

    def step():
        if dist is None:
            return spg.points_sum_compress([partial(0, n)])
        return shard.sharded_msm(dist, partial, n, dev)[0]

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    outs = set()
    for _ in range(a.steps):
        outs.add(step())
    sync()
    dt = time.perf_counter() - t0
    prof = profile_pass(ctx, step, a.steps)
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    assert len(outs) == 1, "MSM result changed between steps"
    lo, hi = shard.chunk(n, rank, world)
    dev_us = sum(v[1] for v in prof.values()) / a.steps
    # algorithmic bytes per point: 32 B scalar + 64 B affine point; the launch sequence of one
    # partial MSM is the unit (the MSM is VALU-bound: mixed additions, reported beside the HBM figure)
    alg = (hi - lo) * 96 + 32
    achieved = alg / (dev_us * 1e-6) / 1e9
    c_win = 16 if hi - lo > 16384 else 8
    madds = (hi - lo) * (253 // c_win + 1)
    roof = {"bound": "hbm", "kernel": "msm (all launches of one partial MSM)", "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "algorithmic_bytes_per_launch": alg, "avg_launch_us": round(dev_us, 1), "launches": a.steps,
            "valu": {"mixed_adds_per_msm": madds, "mixed_adds_per_s": round(madds / (dev_us * 1e-6), 1),
                     "note": "fixed-base signed windows: one 7M mixed addition per nonzero digit"}}
    cpu, bitexact, cpu_verify_ms = None, None, None
    if rank == 0 and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import numpy as np

        import pyoracle  # the checker / CPU baseline only

        pyoracle.build()
        pts = gens.compressed()
        ref_pts = pyoracle.gens_stream(b"spg_bench_msm", n + 1)
        tc = time.perf_counter()
        ref = pyoracle.msm(ref_pts[:n], sc)
        tcpu = time.perf_counter() - tc
        bitexact = bool(np.array_equal(pts, ref_pts) and ref in outs)
        if world == 1:
            cpu = {"value": round(n / tcpu, 1), "unit": "points/s", "cores": 1, "kind": "port",
                   "sample": f"the whole MSM ({n} pairs) by the oracle's vartime Pippenger restatement incl. point "
                             f"decompression, {tcpu:.2f} s on 1 host thread"}
    if rank == 0:
        print(json.dumps({
            "metric": "MSM points/sec (GroupElement::vartime_multiscalar_mul, 2^%d points); result bit-exact" % a.log_msm,
            "value": round(n * a.steps / dt, 1), "unit": "points/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "ristretto255 / fq252",
            "data": "synthetic scalars (splitmix64 seed 1 + edge cases), generators MultiCommitGens(2^k, spg_bench_msm)",
            "config": {"workload": "single MSM, SURVEY 8d config 2", "points": n,
                       "parallelism": f"contiguous shards x{world}, allgather of partials ({backend})"},
            "roofline": roof, "cpu_baseline": cpu, "result_bitexact_vs_cpu": bitexact,
            "result": sorted(outs)[0].hex(), "device_us_per_partial": round(dev_us, 1),
            "kernels": {k: {"launches_per_step": v[0] / a.steps, "us_per_step": round(v[1] / a.steps, 1)}
                        for k, v in sorted(prof.items(), key=lambda kv: -kv[1][1])}}))
    if dist is not None:
        dist.destroy_process_group()


def main_spark(a):
    """SparseMatPolynomial::multi_evaluate + SparseMatPolyEvalProof::prove over the three
    2^k-nonzero matrices (A, B, C) with num_vars_x = num_vars_y = k. A step is one multi_evaluate at (rx, ry)
    plus one full SPARK evaluation proof (derefs, derefs commit, hash layer, product trees, batched layer
    sumchecks, hash-layer PolyEvalProofs) with the dense representation resident in HBM (multi_commit is the
    preprocessing step, SNARK::encode, and is timed separately). Multi-GPU (default --mode shard): ONE proof split
    over the ranks (spg_set_comm; SURVEY 8e: Hyrax rows, interleaved product trees, per-round (e0, e2, e3)
    allgathers over RCCL) -> strong scaling; --mode replicas: an independent proof per rank (weak)."""
    import numpy as np
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
    shard = world > 1 and (a.mode or "shard") == "shard"
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend)
    ndev = torch.cuda.device_count()
    gpu = local % ndev if ndev else local
    if torch.cuda.is_available():
        torch.cuda.set_device(gpu)
    import spg
    import workload

    k = a.log_nnz
    ctx = spg.Context(gpu)
    if shard:
        ctx.set_comm(rank, world, spg.torch_allgather(dist, device=f"cuda:{gpu}" if backend == "nccl" else "cpu"))
    t0 = time.perf_counter()
    wl = workload.SparkWorkload(k)
    views = workload.CViews(wl)
    t_gen = time.perf_counter() - t0
    rng = np.random.default_rng(3 + (0 if shard else rank))
    r = rng.integers(0, 1 << 63, size=(2 * k, 4), dtype=np.uint64)
    r[:, 3] &= np.uint64((1 << 60) - 1)
    rx, ry = r[:k], r[k:]
    t0 = time.perf_counter()
    comm = spg.SparkCommitment(ctx, views.inst, b"gens_r1cs_eval", wl.nnz, 3)
    t_commit = time.perf_counter() - t0
    inst = spg.R1CSInst(ctx, views.inst)
    seed = workload.tape_seed()

    def step():
        evals = spg.r1cs_multi_evaluate(ctx, inst, 1, rx, ry)
        return comm.prove(rx, ry, evals, spg.Transcript(b"spark_bench"), spg.RandomTape(b"proof", seed))

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(a.warmup):
        step()
    sync()
    t0 = time.perf_counter()
    proofs = set()
    for _ in range(a.steps):
        proofs.add(hashlib.sha256(step()).hexdigest())
    sync()
    dt = time.perf_counter() - t0
    prof = profile_pass(ctx, step, a.steps)
    same = None
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        if shard:  # every rank of one sharded proof must hold the same bytes
            hs = [None] * world
            dist.all_gather_object(hs, sorted(proofs))
            same = all(h == hs[0] for h in hs)
    assert len(proofs) == 1, "proof bytes changed between steps"
    nnz = 3 * wl.nnz
    value = nnz * (1 if shard else world) * a.steps / dt
    top = sorted(prof.items(), key=lambda kv: -kv[1][1])[:10]
    kernels = {n: {"launches_per_step": v[0] / a.steps, "ms_per_step": round(v[1] / a.steps / 1e3, 3),
                   "GBps": round(v[2] / (v[1] * 1e-6) / 1e9, 1) if v[2] else None} for n, v in top}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle  # the checker / CPU baseline only

        pyoracle.build()
        kc = min(a.cpu_log_nnz, k)
        wc = workload.SparkWorkload(kc)
        rc_ = rng.integers(0, 1 << 63, size=(2 * kc, 4), dtype=np.uint64)
        rc_[:, 3] &= np.uint64((1 << 60) - 1)
        pyoracle.spark_prove(wc, rc_[:kc], rc_[kc:], seed)
        tcpu = pyoracle.spark_last_prove_us() * 1e-6
        cpu = {"value": round(3 * (1 << kc) / tcpu, 1), "unit": "nonzeros/s", "cores": 1, "kind": "port",
               "sample": f"3 x 2^{kc} nonzeros (same generator), multi_evaluate + SparseMatPolyEvalProof::prove, "
                         f"{tcpu:.2f} s on 1 host thread"}
    if rank == 0:
        print(json.dumps({
            "metric": "SPARK nonzeros/sec (sparse_mlpoly multi_evaluate + SparseMatPolyEvalProof::prove)",
            "value": round(value, 1), "unit": "nonzeros/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if shard else "weak",
            "vs_baseline": None, "dtype": "fq252 (8x u32 Montgomery limbs), ristretto255",
            "data": "synthetic (SURVEY 8d config 5 generator, seed 5)",
            "config": {"workload": "SparseMatPolyEvalProof::prove, batch 3 (src/sparse_mlpoly.rs:1497-1564)",
                       "log_nnz": k, "num_vars_x": k, "num_vars_y": k,
                       "parallelism": f"one proof sharded x{world} ({backend})" if shard else f"replicas x{world}"},
            "roofline": roofline_of(prof, None), "cpu_baseline": cpu, "proof_sha256": sorted(proofs)[0][:16],
            "ranks_agree": same, "commit_s": round(t_commit, 3), "host_gen_s": round(t_gen, 3),
            "device_busy_ms_per_step": round(sum(v[1] for v in prof.values()) / a.steps / 1e3, 3),
            "kernels": kernels}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
