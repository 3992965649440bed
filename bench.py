#!/usr/bin/env python3
"""Benchmark for the MI355X Spartan prover (libspg.so), one JSON line on rank 0.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1 either launched under
torch.distributed.run (WORLD_SIZE must equal N, or the run exits 2 before any work), or started plainly, in which case
bench.py starts the N ranks itself (child processes, env:// rendezvous on 127.0.0.1, one GPU per LOCAL_RANK) before
anything touches a GPU, and rank 0 prints the line.

--workload snark (default, the headline metric): SNARK::prove (src/lib.rs:971-2746)
    on a synthetic 2^20-constraint program (2 block types x 2^9 executions x 2^10 constraints), instances
    encoded and witness resident in HBM before the timed region; every step produces the full bincode(SNARK),
    compared byte-for-byte with the CPU oracle's. Multi-GPU: independent replicas (weak scaling).
    At N = 1 the same line also carries every other single-GPU BASELINE config, each measured in this run with its
    own roofline and CPU baselines (--extras none skips them): config 2 (`config2_msm`: one 2^16-point MSM;
    `config2_rows`: the 1024 x 1024 Hyrax row commit of a 2^20-entry polynomial), config 4 on one GPU
    (`config4_r1cs`: R1CSProof::prove over P = 8 x 2^9 x 2^10 = 2^22 constraints), config 5 (`config5_spark`:
    multi_evaluate + SparseMatPolyEvalProof::prove over 3 x 2^24 nonzeros) and config 1 (`config1_cpu`: the 2^12
    SNARK::prove on the CPU path alone, with the reference's per-phase Timer breakdown).
--workload r1cs: R1CSProof::prove alone (src/r1csproof.rs:210-685); --mode shard splits ONE proof over the ranks
    by instance with a per-round allgather; the shard default is SURVEY 8d config 4's shape, P = 8 instances x 2^9
    executions x 2^10 constraints = 2^22. Sharded modes exchange over libspg's own RCCL transport
    (spg_set_comm_rccl) whenever the backend is nccl; --comm callback selects the torch.distributed callback.
--workload spark: SURVEY 8d config 5 alone; --workload msm: SURVEY 8d config 2 alone (both strong scaling
    over the ranks by default).

Rooflines: `roofline` belongs to the kernel with the most device time that has a work model -- VALU work (curve
mixed additions, one per nonzero signed window digit) against the measured whole-GPU ext_madd throughput, or
algorithmic HBM bytes against 8 TB/s; `roofline_hbm` / `roofline_valu` give the largest kernel of each kind.
Per-launch times are libspg's HIP events on its context stream (spg_prof_read2) in a profiling pass after the
timed steps; `traffic` is the PMC-measured HBM bytes per launch from the committed rocprofv3 summary of the same
workload (TRAFFIC below: scripts/gpu_run.sh PMC=1). `device_busy_ms_per_step` is the union of the timed
intervals, since kernels on the context's second stream overlap those of the main one, without the resident
layer-round launches (their intervals include the host's answers between rounds);
`device_busy_incl_resident_ms_per_step` counts them too.
`cpu_baseline` is the C++ CPU restatement of the reference (oracle/) on rank 0 at N = 1: one thread on the full
workload, and `cpu_baseline_all_cores` the same work run as one independent prove per usable host core at once.
"""
import argparse
import faulthandler
import hashlib
import json
import math
import os
import sys
import threading
import time

# a native fault (libspg, the oracle, the HIP runtime) prints every thread's Python stack on stderr before the process
# dies, so a crash in a driver run names the step it happened in
faulthandler.enable()

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (/opt/skills/guides/MI355X_MICROARCH.md)
# whole-GPU ext_madd throughput at 8 resident 256-thread blocks per CU (3.00e10/s), measured on MI355X by
# scripts/micro/ext_throughput.hip (output: profiles/r03_ext_throughput.txt)
MADD_PEAK = 3.0e10
# issue-rate ceiling of the same addition: ext_madd compiles to 1,527 VALU instructions per lane-addition (511 of them
# v_mad_u64_u32; `hipcc -S` of scripts/micro/ext_throughput.hip, k_thr<2> loop body); 1,024 SIMDs issuing one wave64
# VALU instruction per 2 cycles at 2.4 GHz bound it at 1024 * 2.4e9 / (2 * 1527) * 64 = 5.15e10 madd/s if every
# instruction were full rate -- an upper bound (64-bit multiply-adds are not), of which MADD_PEAK is 0.58
MADD_ISSUE_CEILING = 1024 * 2.4e9 / (2 * 1527) * 64
# whole-GPU throughput of the device Fq product (fq_mul_ps, the scalar field's Montgomery product) with 4 independent
# chains per lane and 8 resident 256-thread blocks per CU: 1.44e11/s, measured on MI355X by
# scripts/micro/fq_throughput.hip (output: profiles/r05_fq_throughput.txt) -- the peak the Fq-product-bound kernels
# (R1CSProof sumcheck evaluations, SPARK layer rounds) are priced against in `roofline_fq`
FQ_PEAK = 1.44e11
GENS_LABEL = b"gens_r1cs_sat"
GENS_NUM_VARS = 1 << 24  # TOTAL_NUM_VARS_BOUND = 10^7 -> 2^24 (examples/interface.rs:557-563)
CONFIGS = {
    # name: (num_cons per instance, num_proofs per instance, witness sections)
    "r1cs_2e20": ([1024, 1024], [512, 512], 1),
    "r1cs_2e16": ([1024, 1024], [32, 32], 1),
    "r1cs_2e22_p8": ([1024] * 8, [512] * 8, 1),
}
# per-launch HBM bytes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_traffic.py) of each workload's own
# run: a kernel's traffic depends on its launch size, so one workload's figures are never reported for another
TRAFFIC = {w: os.path.join(ROOT, "profiles", f) for w, f in (
    ("snark", "r06_pmc_traffic.json"), ("msm16", "r05_pmc_traffic_msm_2e16.json"),
    ("spark24", "r05_pmc_traffic_spark_2e24.json"), ("rows", "r05_pmc_traffic_rows_1024.json"),
    ("r1cs22", "r06_pmc_traffic_r1cs_2e22.json"))}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="r1cs workload shape (default: r1cs_2e22_p8 with --mode shard, else r1cs_2e20)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", default=None, choices=["replicas", "shard"],
                    help="N > 1: replicas (independent proofs per rank) or shard (one proof split over the ranks); "
                         "default: shard for --workload spark / msm, replicas otherwise")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl with a GPU)")
    ap.add_argument("--log-msm", type=int, default=16, help="msm: 2^k (scalar, generator) pairs")
    ap.add_argument("--workload", default="snark", choices=["snark", "r1cs", "spark", "msm", "rows", "launchcheck"],
                    help="snark: the headline metric (SNARK::prove, SURVEY 8d config 3); r1cs: its block "
                         "R1CSProof::prove alone; spark: SURVEY 8d config 5 (SPARK); msm: config 2; rows: config 2's "
                         "1024 x 1024 row batch")
    ap.add_argument("--log-cons", type=int, default=10, help="snark: 2^k constraints per block")
    ap.add_argument("--log-proofs", type=int, default=9, help="snark: 2^k executions per block")
    ap.add_argument("--log-nnz", type=int, default=24, help="spark: 2^k nonzeros per matrix (x3 matrices)")
    ap.add_argument("--cpu-log-nnz", type=int, default=16, help="spark: CPU baseline sample size")
    ap.add_argument("--extras-log-nnz", type=int, default=24,
                    help="snark: config 5's 2^k nonzeros per matrix in the extras (24 = BASELINE config 5; smaller only "
                         "for rehearsals with several ranks on one GPU)")
    ap.add_argument("--extras", default="msm,rows,r1cs,spark,cpu1",
                    help="snark at N = 1: the other BASELINE configs measured in the same run "
                         "(msm, rows, r1cs, spark, cpu1; 'none')")
    ap.add_argument("--comm", default="auto", choices=["auto", "rccl", "callback"],
                    help="sharded modes: libspg's RCCL transport (auto: with the nccl backend) or the torch callback")
    ap.add_argument("--traffic", default=None, help="per-launch HBM bytes from rocprofv3 --pmc (scripts/pmc_traffic.py)")
    return ap.parse_args()


# ---------------------------------------------------------------- shared plumbing
class Env:
    """one process per GPU (torchrun env), torch.distributed only for the barrier / max-over-ranks timer and the
    allgather of the sharded modes"""

    def __init__(self, a):
        import torch

        self.torch = torch
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = a.backend or ("nccl" if torch.cuda.is_available() else "gloo")
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist

            # the gloo library reports its connections on stdout; the bench's stdout carries one JSON line only, so
            # the process group comes up (and connects, at its first barrier) with fd 1 pointed at stderr
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group(self.backend)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist
        ndev = torch.cuda.device_count()
        self.ndev = ndev
        if ndev and self.world > ndev and "SPG_COMB_GB" not in os.environ:
            # a rehearsal with several ranks on one GPU: each process's comb tables get a share of the HBM (libspg reads
            # the cap at its first table), so every rank keeps room for its workspaces; results are the same bytes
            os.environ["SPG_COMB_GB"] = str(max(16, 96 // -(-self.world // ndev)))
        self.gpu = self.local % ndev if ndev else self.local  # ranks share a GPU only in rehearsals
        if torch.cuda.is_available():
            torch.cuda.set_device(self.gpu)
        self.comm_device = f"cuda:{self.gpu}" if self.backend == "nccl" else "cpu"

    def sync(self):
        if self.torch.cuda.is_available():
            self.torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, x):
        if self.dist is None:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64,
                              device="cuda" if self.torch.cuda.is_available() else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def install_comm(env, ctx, how="auto"):
    """the exchange transport of a sharded call: libspg's own RCCL communicator (spg_set_comm_rccl: ncclAllGather on
    the context's stream over xGMI, no Python per exchange) with the nccl backend, else the torch.distributed
    callback (spg_set_comm); returns the transport's name"""
    import spg

    if how == "rccl" or (how == "auto" and env.backend == "nccl"):
        ctx.set_comm_rccl(env.rank, env.world, env.dist)
        return "rccl (spg_set_comm_rccl)"
    ctx.set_comm(env.rank, env.world, spg.torch_allgather(env.dist, device=env.comm_device))
    return f"callback (torch.distributed {env.backend})"


def timed(env, step, steps, warmup):
    """warmup untimed steps, then `steps` timed ones bracketed by barrier + synchronize; returns (seconds max over
    ranks, per-step laps on this rank, set of result hashes)"""
    for _ in range(warmup):
        step()
    env.sync()
    t0 = time.perf_counter()
    res, laps = [], []
    for _ in range(steps):
        t1 = time.perf_counter()
        res.append(step())
        laps.append(time.perf_counter() - t1)
    env.sync()
    dt = time.perf_counter() - t0
    # the determinism check (every step's bytes hashed) is the bench's own bookkeeping: after the timed region
    return env.max_over_ranks(dt), laps, {hashlib.sha256(r).hexdigest() for r in res}


def profile_pass(ctx, step, steps):
    """per-kernel HIP-event timing (libspg spg_prof_read2) of `steps` extra steps run after the timed region, so
    the events never perturb `value`; returns {kernel: (launches, us, algorithmic bytes, VALU madds)} summed"""
    ctx.prof_enable(True)
    ctx.prof_read(reset=True)
    for _ in range(steps):
        step()
    prof = Prof(ctx.prof_read(reset=True, ops=True))
    ctx.prof_enable(False)
    busy = prof.pop("(device_busy)", None)
    res = prof.pop("(device_busy_resident)", None)
    prof.busy_us = busy[1] if busy else sum(v[1] for v in prof.values())
    prof.busy_resident_us = res[1] if res else prof.busy_us
    return prof


class Prof(dict):
    """per-kernel timings of a profile pass; busy_us = the device's busy time (union of the timed intervals: kernels
    of the context's second stream overlap the main stream's, so the per-kernel sum overstates it), leaving out the
    resident launches (spark_layer_persist: their interval spans the host's answers between rounds);
    busy_resident_us = the union with them"""
    busy_us = 0.0
    busy_resident_us = 0.0


# scopes that share a device kernel with another scope: the PMC passes name the kernel (scripts/pmc_traffic.py), and a
# workload's own traffic file holds only its own launches of it
SCOPE_KERNEL = {"msm_comb_single": "msm_comb"}


def traffic_of(kernel, traffic_file):
    if traffic_file and os.path.exists(traffic_file):
        tr = json.load(open(traffic_file)).get("kernels", {})
        for k in (kernel, SCOPE_KERNEL.get(kernel)):
            if k in tr:
                return tr[k]["hbm_bytes_per_launch"]
    return None


def roofline_hbm(prof, traffic_file=None):
    """HBM roofline of the modelled-bytes kernel with the largest device time"""
    cand = {k: v for k, v in prof.items() if v[2] > 0}
    if not cand:
        return None
    dom = max(cand, key=lambda k: cand[k][1])
    launches, us, nbytes = cand[dom][:3]
    per = nbytes / launches
    achieved = per / (us / launches * 1e-6) / 1e9
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic_of(dom, traffic_file),
            "algorithmic_bytes_per_launch": per, "avg_launch_us": us / launches, "launches": launches,
            # a launch that moves < 64 MB cannot approach the HBM peak behind a ~4 us small-launch floor: its regime
            # is the round-trip latency (transcript-sequential rounds over KB-sized vectors), DESIGN.md 4
            "regime": "bandwidth" if per >= (64 << 20) else "latency"}


def roofline_valu(prof, traffic_file=None):
    """VALU roofline of the modelled-madds kernel with the largest device time: curve mixed additions per second
    against the measured whole-GPU ext_madd throughput"""
    cand = {k: v for k, v in prof.items() if len(v) > 3 and v[3] > 0}
    if not cand:
        return None
    dom = max(cand, key=lambda k: cand[k][1])
    launches, us, nbytes, ops = cand[dom][:4]
    achieved = ops / (us * 1e-6)
    traffic = traffic_of(dom, traffic_file)
    out = {"bound": "valu", "kernel": dom, "achieved": round(achieved, 1), "peak": MADD_PEAK, "unit": "ext_madd/s",
           "frac": round(achieved / MADD_PEAK, 5), "traffic": traffic,
           "algorithmic_madds_per_launch": ops / launches, "avg_launch_us": us / launches, "launches": launches,
           "peak_source": "measured whole-GPU ext_madd throughput, scripts/micro/ext_throughput.hip, 8 blocks/CU "
                          "(profiles/r03_ext_throughput.txt)",
           "issue_rate_ceiling": round(MADD_ISSUE_CEILING, 1),
           "frac_of_issue_ceiling": round(achieved / MADD_ISSUE_CEILING, 5)}
    if nbytes:  # the kernel's table reads are modelled too: its traffic against them
        out["algorithmic_bytes_per_launch"] = nbytes / launches
        if traffic:
            out["traffic_over_algorithmic"] = round(traffic / (nbytes / launches), 3)
    return out


def roofline_fq(prof, traffic_file=None):
    """VALU roofline of the modelled-Fq-products kernel with the largest device time: scalar-field products per
    second (DESIGN.md 3.9 per-launch models) against the measured whole-GPU fq_mul throughput, beside the same launches'
    algorithmic HBM rate"""
    cand = {k: v for k, v in prof.items() if len(v) > 4 and v[4] > 0}
    if not cand:
        return None
    dom = max(cand, key=lambda k: cand[k][1])
    launches, us, nbytes, _, fqm = cand[dom][:5]
    achieved = fqm / (us * 1e-6)
    out = {"bound": "valu_fq", "kernel": dom, "achieved": round(achieved, 1), "peak": FQ_PEAK, "unit": "Fq products/s",
           "frac": round(achieved / FQ_PEAK, 5), "traffic": traffic_of(dom, traffic_file),
           "algorithmic_fq_products_per_launch": fqm / launches, "avg_launch_us": us / launches, "launches": launches,
           "peak_source": "measured whole-GPU fq_mul throughput, scripts/micro/fq_throughput.hip, ILP 4, 8 blocks/CU "
                          "(profiles/r05_fq_throughput.txt)"}
    if nbytes:
        gbs = nbytes / launches / (us / launches * 1e-6) / 1e9
        out["algorithmic_bytes_per_launch"] = nbytes / launches
        out["hbm_GBps"] = round(gbs, 1)
        out["hbm_frac"] = round(gbs / HBM_PEAK_GBS, 5)
    return out


def rooflines(prof, traffic_file=None):
    """(roofline of the kernel with the most device time among the modelled ones, hbm one, valu one)"""
    h, v = roofline_hbm(prof, traffic_file), roofline_valu(prof, traffic_file)
    if h is None or v is None:
        return (h or v), h, v
    th = prof[h["kernel"]][1]
    tv = prof[v["kernel"]][1]
    return (v if tv >= th else h), h, v


def kernel_table(prof, steps, top=10):
    rows = sorted(prof.items(), key=lambda kv: -kv[1][1])[:top]
    return {k: {"launches_per_step": v[0] / steps, "ms_per_step": round(v[1] / steps / 1e3, 3),
                "GBps": round(v[2] / (v[1] * 1e-6) / 1e9, 1) if v[2] else None,
                "madds_per_s": round(v[3] / (v[1] * 1e-6), 1) if len(v) > 3 and v[3] else None,
                "fq_products_per_s": round(v[4] / (v[1] * 1e-6), 1) if len(v) > 4 and v[4] else None}
            for k, v in rows}


def usable_cores():
    """host CPUs this process may use: the affinity mask, capped by the cgroup quota and OMP_NUM_THREADS (the GPU
    box sets it to the job's CPU share)"""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def run_threads(fn, k):
    """fn() on k threads at once (the oracle's ctypes calls release the GIL); returns the wall seconds"""
    errs = []

    def body():
        try:
            fn()
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=body) for _ in range(k)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    return time.perf_counter() - t0


def oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # the checker / CPU baseline only

    pyoracle.build()
    return pyoracle


def all_cores_baseline(fn, units, unit, sample):
    """the same CPU work as one independent oracle run per usable core, concurrently: units x k / wall"""
    k = usable_cores()
    dt = run_threads(fn, k)
    return {"value": round(units * k / dt, 1), "unit": unit, "cores": k, "kind": "port",
            "sample": f"{k} concurrent independent copies of: {sample}; {dt:.2f} s wall"}


def precomputation(c0, c1, note):
    """the fixed-base tables a workload built (spg_comb_stats before / after its first steps): comb tables' HBM bytes
    and build seconds, and the 2^k G_i tables of every live generator set"""
    return {"comb_table_bytes": c1[0] - c0[0], "comb_tables_built": c1[1] - c0[1],
            "comb_build_s": round(c1[2] - c0[2], 4), "gens_table_bytes_process": c1[3], "note": note}


def no_table_leg(env, ctx, step, steps, warmup, outs):
    """the same steps with this context's comb tables switched off (spg_set_comb 0: the bucket Pippenger pipelines
    over the 2^k G_i tables), so the MSM comparison with the CPU's table-free vartime Pippenger can be read like for
    like; the result must be the same bytes"""
    ctx.set_comb(False)
    try:
        got = set()

        def st():
            r = step()
            got.add(r if isinstance(r, bytes) else r.tobytes())
            return r if isinstance(r, bytes) else r.tobytes()

        dt, laps, _ = timed(env, st, steps, warmup)
    finally:
        ctx.set_comb(True)
    return {"ms_per_step": round(dt / steps * 1e3, 3), "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3),
            "same_result": got == outs, "path": "bucket Pippenger over the 2^k G_i tables (spg_set_comb 0)"}


# ---------------------------------------------------------------- SNARK::prove (headline, config 3)
def main_snark(a):
    """The headline metric: SNARK::prove (src/lib.rs:971-2746) on the synthetic program of
    workload.SnarkWorkload: 2 block types x 2^log_proofs executions x 2^log_cons constraints (N = 2^20 by
    default), no memory operations, vars_gens = R1CSGens(gens_r1cs_sat, 2^24). A step is one full SNARK::prove
    (witness recurrences, every Hyrax commitment, the block / pairwise / perm-root R1CSProofs with their
    R1CSEvalProofs, perm-product, shift and IO proofs) with the instances encoded (SNARK::encode, preprocessing)
    and block_vars / exec inputs resident in HBM. Multi-GPU: independent replicas (one SNARK per rank)."""
    env = Env(a)
    import spg
    import workload

    ctx = spg.Context(env.gpu)
    t0 = time.perf_counter()
    wl = workload.SnarkWorkload(num_blocks=2, log_cons=a.log_cons, log_proofs=a.log_proofs,
                                num_vars=1 << a.log_cons, seed=0x5350415254414E31 + env.rank)
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

    def prove(w):
        return spg.snark_prove(ctx, block, pairwise, perm_root, w, gens, spg.Transcript(b"snark_bench"),
                               spg.RandomTape(b"proof", seed))

    comb0 = spg.comb_stats()
    dt, laps, proofs = timed(env, lambda: prove(wit), a.steps, a.warmup)
    assert len(proofs) == 1, "proof bytes changed between steps"
    comb1 = spg.comb_stats()
    # the drop-in mode: every append / challenge of the prove goes through C callbacks
    # into a caller-owned merlin transcript (libspg_hostcheck's native merlin, as a Rust caller's extern "C" trampolines
    # over &mut Transcript would) instead of libspg's own; same steps, timed the same way, right after the timed region
    def prove_cb(w):
        return spg.snark_prove(ctx, block, pairwise, perm_root, w, gens, spg.Transcript.from_native_merlin(b"snark_bench"),
                               spg.RandomTape(b"proof", seed))

    dt_cb, laps_cb, proofs_cb = timed(env, lambda: prove_cb(wit), a.steps, 1)
    # the two modes alternated step by step (box drift cancels): medians of each
    alt = {0: [], 1: []}
    for i in range(2 * a.steps):
        t1 = time.perf_counter()
        (prove_cb if i % 2 else prove)(wit)
        alt[i % 2].append(time.perf_counter() - t1)
    med_native, med_cb = (sorted(alt[m])[len(alt[m]) // 2] for m in (0, 1))
    prof = profile_pass(ctx, lambda: prove(wit), a.steps)
    # per-call input work of a drop-in SNARK::prove (it receives Vec<Vec<VarsAssignment>> on every call): the
    # witness upload (spg_snark_witness_new, PCIe + io-row parsing) + the prove, median of 5 (beside value)
    incl = []
    for _ in range(5):
        t1 = time.perf_counter()
        proof = prove(spg.SnarkWitness(ctx, views.inputs))
        incl.append(time.perf_counter() - t1)
    t_incl = sorted(incl)[len(incl) // 2]
    # SNARK::verify of the same proof on the product path (not part of value; reported beside it)
    verify_ok, _ = spg.snark_verify(ctx, block, pairwise, perm_root, views.inputs, gens, spg.Transcript(b"snark_bench"),
                                    proof)
    t1 = time.perf_counter()
    for _ in range(3):
        spg.snark_verify(ctx, block, pairwise, perm_root, views.inputs, gens, spg.Transcript(b"snark_bench"), proof)
    t_verify = (time.perf_counter() - t1) / 3
    N = wl.total_constraints
    value = N * env.world * a.steps / dt
    roof, roof_h, roof_v = rooflines(prof, a.traffic or TRAFFIC["snark"])
    cpu = cpu_all = bitexact = cpu_verify_ms = None
    if env.rank == 0 and env.world == 1 and not a.no_cpu_baseline:
        po = oracle()
        ref, rc = po.snark_prove(wl, seed, gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS, label=b"snark_bench")
        tcpu = po.snark_last_prove_us() * 1e-6
        cpu_verify_ms = po.snark_last_verify_us() * 1e-3
        cpu = {"value": round(N / tcpu, 1), "unit": "constraints/s", "cores": 1, "kind": "port",
               "sample": f"full workload ({N} constraints), one SNARK::prove (instances pre-encoded), "
                         f"{tcpu:.2f} s on 1 host thread; oracle verifier status {rc}"}
        bitexact = hashlib.sha256(ref).hexdigest() in proofs
        # all cores: one oracle copy per usable core encodes and derives its generators, all meet at a barrier, then
        # all prove at once; the wall time runs from the first prove's start to the last one's end (SNARK::prove alone,
        # like the GPU step: encode, R1CSGens and verification outside)
        k_all = usable_cores()
        dt_all = po.snark_concurrent_prove(wl, seed, k_all, gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS,
                                           label=b"snark_bench")
        cpu_all = {"value": round(N * k_all / dt_all, 1), "unit": "constraints/s", "cores": k_all, "kind": "port",
                   "sample": f"{k_all} concurrent independent copies of the full workload's SNARK::prove ({N} "
                             f"constraints each), proving together after a barrier (prove only); {dt_all:.2f} s wall "
                             f"from the first prove's start to the last one's end"}
    extras = {}
    want = set(a.extras.split(",")) if a.extras != "none" else set()
    if env.world > 1:
        # N > 1: the BASELINE configs that shard, each as ONE proof split over the ranks with libspg's exchanges
        # (RCCL under the nccl backend), strong scaling; every rank must end with the same bytes (ranks_agree), and the
        # bytes equal the N = 1 line's config4_r1cs / config5_spark (same workload seeds). Measured after the replicas.
        if "r1cs" in want:
            extras["config4_r1cs"] = guarded(lambda: r1cs_core(env, ctx, "r1cs_2e22_p8", True, 5, 1, False,
                                                               TRAFFIC["r1cs22"], a.comm), env)
        if "spark" in want:
            extras["config5_spark"] = guarded(lambda: spark_core(env, ctx, a.extras_log_nnz, a.cpu_log_nnz, 5, 1, "shard",
                                                                 False, TRAFFIC["spark24"] if a.extras_log_nnz == 24
                                                                 else None, a.comm), env)
    if env.world == 1 and want:
        cpu_on = not a.no_cpu_baseline
        if "msm" in want:
            extras["config2_msm"] = guarded(lambda: msm_core(env, ctx, 16, a.steps, a.warmup, cpu_on, TRAFFIC["msm16"]))
        if "rows" in want:
            extras["config2_rows"] = guarded(lambda: rows_core(env, ctx, a.steps, a.warmup, cpu_on, TRAFFIC["rows"]))
        if "r1cs" in want:
            extras["config4_r1cs"] = guarded(lambda: r1cs_core(env, ctx, "r1cs_2e22_p8", False, 5, 1, cpu_on,
                                                               TRAFFIC["r1cs22"]))
        if "spark" in want:
            extras["config5_spark"] = guarded(lambda: spark_core(env, ctx, a.extras_log_nnz, a.cpu_log_nnz, 5, 1,
                                                                 "replicas", cpu_on, TRAFFIC["spark24"]
                                                                 if a.extras_log_nnz == 24 else None))
        if "cpu1" in want and cpu_on:
            extras["config1_cpu"] = guarded(cpu1_core)
    if env.rank == 0:
        out = {
            "metric": "R1CS constraints/sec (SNARK::prove) at 2^20 vars; proof bytes bit-exact",
            "value": round(value, 1), "unit": "constraints/s", "n_gpus": env.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fq252 (8x u32 Montgomery limbs), ristretto255",
            "data": "synthetic program (2 block types, chain-of-squarings blocks, seeded), random-tape seed fixed",
            "config": {"workload": "SNARK::prove (src/lib.rs:971-2746)", "block_types": 2,
                       "constraints_per_block": 1 << a.log_cons, "executions_per_block": 1 << a.log_proofs,
                       "constraints_per_gpu": N, "num_vars": wl.num_vars, "num_ios": wl.num_ios,
                       "gens": "R1CSGens(gens_r1cs_sat, 2^24)", "parallelism": f"replicas x{env.world}",
                       "devices_visible": env.ndev, "ranks_share_a_gpu": env.world > env.ndev,
                       "launcher": os.environ.get("SPG_BENCH_LAUNCHER") or ("torchrun" if env.world > 1 else None)},
            "roofline": roof, "roofline_hbm": roof_h, "roofline_valu": roof_v,
            "roofline_fq": roofline_fq(prof, a.traffic or TRAFFIC["snark"]),
            "cpu_baseline": cpu, "cpu_baseline_all_cores": cpu_all, "proof_bitexact_vs_cpu": bitexact,
            "proof_sha256": sorted(proofs)[0][:16],
            "device_busy_ms_per_step": round(prof.busy_us / a.steps / 1e3, 3),
            "device_busy_incl_resident_ms_per_step": round(prof.busy_resident_us / a.steps / 1e3, 3),
            "value_incl_witness_upload": round(N * env.world / t_incl, 1),
            "ms_per_step_incl_witness_upload": round(t_incl * 1e3, 3),
            "transcript_mode": {
                "value": "native (libspg's own merlin transcript)",
                "callback": {"transcript": "caller-owned merlin behind spg_transcript_new_callbacks (C callbacks, "
                                           "libspg_hostcheck spgh_merlin_*)",
                             "value": round(N * env.world * a.steps / dt_cb, 1),
                             "ms_per_step": round(dt_cb / a.steps * 1e3, 3),
                             "ms_per_step_median": round(sorted(laps_cb)[len(laps_cb) // 2] * 1e3, 3),
                             "over_native": round(dt_cb / dt, 4), "same_bytes": proofs_cb == proofs,
                             "alternated": {"native_ms_median": round(med_native * 1e3, 3),
                                            "callback_ms_median": round(med_cb * 1e3, 3),
                                            "over_native": round(med_cb / med_native, 4)}}},
            "precomputation": precomputation(
                comb0, comb1, "fixed-base tables over the public generators, built once per generator set on first use "
                              "(in the warmup steps here, outside value) and kept in HBM; the reference's SNARK::prove "
                              "runs vartime MSMs without tables"),
            "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3),
            "ms_per_step_min": round(min(laps) * 1e3, 3), "verify_ms": round(t_verify * 1e3, 2),
            "ms_per_step_laps": [round(x * 1e3, 2) for x in laps],
            "verify_ok": verify_ok, "cpu_verify_ms_1thread": None if cpu_verify_ms is None else round(cpu_verify_ms, 1),
            "encode_s": round(t_encode, 3), "host_gen_s": round(t_gen, 3), "kernels": kernel_table(prof, a.steps),
        }
        out.update(extras)
        print(json.dumps(out))
    env.close()


def guarded(fn, env=None):
    """an extra config's result, or the error it raised (the headline line is printed either way). With several ranks
    (env given) the ranks exchange a failure flag after fn. That keeps them in step when every rank fails together --
    libspg's own exchanges fail all ranks at once (status-framed allgathers) -- or when a rank fails before fn's first
    collective. A rank that fails between two of fn's torch collectives (the barrier or max-over-ranks of timed(), the
    all_gather_object of the rank check) meets the others' next collective with this flag exchange instead; that can
    hang or raise in the backend, and the launcher (or the driver's time limit) then ends the run: the guarantee does
    not extend to that case."""
    try:
        out, err = fn(), None
    except Exception as e:  # noqa: BLE001
        out, err = None, {"error": repr(e)[:500]}
    if env is not None and env.dist is not None:
        bad = env.max_over_ranks(1.0 if err else 0.0)
        if bad and not err:
            err = {"error": "another rank failed in this config"}
    return err or out


# ---------------------------------------------------------------- R1CSProof::prove (config 4)
def r1cs_core(env, ctx, cfg, shard, steps, warmup, cpu_on, traffic_file=None, comm="auto"):
    """R1CSProof::prove (src/r1csproof.rs:210-685) on the CONFIGS shape `cfg`. shard: ONE proof split over the ranks by
    instance, its per-round (e0, e2, e3) sums and the final gathers over the ranks (RCCL with the nccl
    backend) -> strong scaling; else an independent proof per rank (weak). A step is one whole proof with the witness
    resident in HBM. CPU baselines (rank 0, N = 1): the oracle on the full workload on 1 host thread (its bytes are
    also the bit-exactness check), and one independent oracle proof per usable core on a 2^6-execution sample."""
    import spg
    import workload

    nc, npf, nws = CONFIGS[cfg]
    transport = None
    if shard:
        p0, p1 = spg.shard_range(len(nc), env.rank, env.world)
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, instances=range(p0, p1))
        transport = install_comm(env, ctx, comm)
    else:
        p0 = p1 = None
        wl = workload.R1CSWorkload(nc, npf, num_sections=nws, seed=0x5350415254414E31 + env.rank,
                                   instances=range(len(nc)))
    seed = workload.tape_seed()
    gens = spg.R1CSGens(ctx, GENS_LABEL, GENS_NUM_VARS)
    views = workload.CViews(wl)
    inst = spg.R1CSInst(ctx, views.inst)

    def upload():
        return spg.R1CSWitness(ctx, views.secs, wl.nws, shard=(p0, p1) if shard else None)

    wit = upload()
    c0 = spg.comb_stats()

    def step():
        pf, _ = spg.r1cs_prove(ctx, gens, inst, wit, wl.P, wl.max_num_proofs, wl.num_proofs, wl.max_num_inputs,
                               wl.num_inputs, spg.Transcript(b"r1cs_bench"), spg.RandomTape(b"proof", seed))
        return pf

    dt, laps, proofs = timed(env, step, steps, warmup)
    pre = precomputation(c0, spg.comb_stats(), "comb tables over R1CSGens' generators, built in the first (warmup) "
                                               "proof and kept in HBM; the CPU baseline uses no tables")
    if not shard:
        assert len(proofs) == 1, "proof bytes changed between steps"
    prof = profile_pass(ctx, step, steps)
    # PCIe-inclusive variant (reported beside value): a drop-in R1CSProof::prove gets its witness in host memory on every
    # call, so each of 3 timed calls uploads it (spg_r1cs_witness_new: streamed, returns once the host buffers are read)
    # and proves; the previous witness is freed first, as a caller dropping it would (its device buffer is reused)
    incl, t_new = [], []
    for _ in range(3):
        wit = None
        t1 = time.perf_counter()
        wit = upload()
        t_new.append(time.perf_counter() - t1)
        step()
        incl.append(time.perf_counter() - t1)
    t_incl = sorted(incl)[1]
    same = None
    if shard:  # every rank of one sharded proof must hold the same bytes, the same in every step
        hs = [None] * env.world
        env.dist.all_gather_object(hs, sorted(proofs))
        same = all(h == hs[0] for h in hs) and len(hs[0]) == 1
        ctx.set_comm(0, 1)
    N = wl.total_constraints  # one proof's constraints (the whole sharded proof, or one replica's)
    units = N if shard else N * env.world
    roof, roof_h, roof_v = rooflines(prof, traffic_file)
    cpu = cpu_all = bitexact = None
    if env.rank == 0 and env.world == 1 and cpu_on:
        po = oracle()
        ref, _ = po.r1cs_prove(wl, seed, gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS, label=b"r1cs_bench")
        tcpu = po.last_prove_seconds()  # R1CSProof::prove alone (R1CSGens derivation outside, like the GPU step)
        cpu = {"value": round(N / tcpu, 1), "unit": "constraints/s", "cores": 1, "kind": "port",
               "sample": f"full workload ({N} constraints), one R1CSProof::prove (prove only), {tcpu:.2f} s on 1 host "
                         f"thread"}
        bitexact = hashlib.sha256(ref).hexdigest() in proofs
        ks = 6  # all cores: a 2^6-execution sample of the same shape per core
        ws = workload.R1CSWorkload(nc, [min(x, 1 << ks) for x in npf], num_sections=nws, instances=range(len(nc)))
        k_all = usable_cores()
        dt_all = po.r1cs_concurrent_prove(ws, seed, k_all, gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS,
                                          label=b"r1cs_bench")
        cpu_all = {"value": round(ws.total_constraints * k_all / dt_all, 1), "unit": "constraints/s", "cores": k_all,
                   "kind": "port",
                   "sample": f"{k_all} concurrent independent copies of R1CSProof::prove of {ws.P} instances x 2^{ks} "
                             f"executions x {nc[0]} constraints ({ws.total_constraints} constraints each; the GPU line "
                             f"proves {N}), proving together after a barrier (prove only); {dt_all:.2f} s wall"}
    return {
        "metric": "R1CS constraints/sec (R1CSProof::prove, data-parallel)", "value": round(units * steps / dt, 1),
        "unit": "constraints/s", "n_gpus": env.world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 3), "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3),
        "higher_is_better": True, "scaling": "strong" if shard else "weak",
        "dtype": "fq252 (8x u32 Montgomery limbs), ristretto255",
        "data": "synthetic (chain-of-squarings R1CS, seeded), random-tape seed fixed",
        "config": {"workload": "R1CSProof::prove (src/r1csproof.rs:210-685)", "shape": cfg, "num_instances": len(nc),
                   "num_cons": nc[0], "num_proofs": npf[0], "witness_sections": nws, "constraints": N,
                   "gens": "R1CSGens(gens_r1cs_sat, 2^24)",
                   "parallelism": f"instance-sharded single proof x{env.world} ({transport})" if shard
                   else f"replicas x{env.world}"},
        "roofline": roof, "roofline_hbm": roof_h, "roofline_valu": roof_v,
        "roofline_fq": roofline_fq(prof, traffic_file), "cpu_baseline": cpu,
        "cpu_baseline_all_cores": cpu_all, "proof_bitexact_vs_cpu": bitexact, "proof_sha256": sorted(proofs)[0][:16],
        "ranks_agree": same, "transport": transport, "device_busy_ms_per_step": round(prof.busy_us / steps / 1e3, 3),
        "precomputation": pre,
        "value_incl_witness_upload": round(units / t_incl, 1), "ms_per_step_incl_witness_upload": round(t_incl * 1e3, 3),
        "witness_new_ms": round(sorted(t_new)[1] * 1e3, 3), "kernels": kernel_table(prof, steps)}


def main_r1cs(a):
    env = Env(a)
    import spg

    shard = (a.mode or "replicas") == "shard" and env.world > 1
    cfg = a.config or ("r1cs_2e22_p8" if shard else "r1cs_2e20")
    ctx = spg.Context(env.gpu)
    out = r1cs_core(env, ctx, cfg, shard, a.steps, a.warmup, not a.no_cpu_baseline,
                    a.traffic or (TRAFFIC["r1cs22"] if cfg == "r1cs_2e22_p8" else None), a.comm)
    if env.rank == 0:
        out["vs_baseline"] = None
        print(json.dumps(out))
    env.close()


# ---------------------------------------------------------------- Hyrax row commit (config 2's row batch)
def rows_core(env, ctx, steps, warmup, cpu_on, traffic_file=None, log_rows=10, log_width=10):
    """SURVEY 8d config 2, second shape: DensePolynomial::commit_inner (src/dense_mlpoly.rs:184-212) of a
    2^20-entry polynomial as 2^10 row MSMs of 2^10 scalars each (the block-witness commit of every config-3 prove),
    generators MultiCommitGens(1024, spg_bench_rows), scalars resident in HBM. A step is the whole batch ending in
    the 1024 compressed row commitments on the host."""
    import numpy as np

    import spg
    import workload

    L, R = 1 << log_rows, 1 << log_width
    gens = spg.Gens(ctx, R, b"spg_bench_rows")
    v, _ = workload.random_fq(L * R, 7)
    Z = workload.to_mont_limbs([int(x) for x in v])
    zbuf = spg.Buf(ctx, Z)
    outs = set()

    def step():
        r = gens.commit_rows_buf(zbuf, L, R)
        outs.add(r.tobytes())
        return r.tobytes()

    c0 = spg.comb_stats()
    dt, laps, _ = timed(env, step, steps, warmup)
    assert len(outs) == 1, "row commitments changed between steps"
    pre = precomputation(c0, spg.comb_stats(), "comb table of MultiCommitGens(1024, spg_bench_rows), built in the first "
                                               "(warmup) step and kept in HBM; the CPU baseline uses no tables")
    no_tab = no_table_leg(env, ctx, step, steps, warmup, outs)
    prof = profile_pass(ctx, step, steps)
    roof, roof_h, roof_v = rooflines(prof, traffic_file)
    dev_us = prof.busy_us / steps
    madds = sum(v[3] for v in prof.values()) / steps
    cpu = cpu_all = bitexact = None
    rows = np.frombuffer(sorted(outs)[0], dtype=np.uint8).reshape(L, 32)
    if env.rank == 0 and cpu_on:
        po = oracle()
        pts = gens.compressed()
        ref_pts = po.gens_stream(b"spg_bench_rows", R + 1)
        ls = 64  # 1-thread sample: the first 64 rows (every row is an independent MSM of the same width)
        tc = time.perf_counter()
        ref = po.commit_rows(ref_pts[:R], ref_pts[R].tobytes(), Z[: ls * R], ls, R)
        tcpu = time.perf_counter() - tc
        bitexact = bool(np.array_equal(pts, ref_pts) and np.array_equal(ref, rows[:ls]))
        cpu = {"value": round(ls * R / tcpu, 1), "unit": "points/s", "cores": 1, "kind": "port",
               "sample": f"{ls} of the {L} rows ({ls} x {R} scalars; their bytes are the bit-exactness check) by the "
                         f"oracle's Pippenger restatement, {tcpu:.2f} s on 1 host thread"}
        cpu_all = all_cores_baseline(lambda: po.commit_rows(ref_pts[:R], ref_pts[R].tobytes(), Z[: ls * R], ls, R),
                                     ls * R, "points/s", f"{ls} rows x {R} scalars by the oracle's Pippenger")
    return {
        "metric": "Hyrax row-commit points/sec (DensePolynomial::commit_inner, 2^%d rows x 2^%d)" % (log_rows, log_width),
        "value": round(L * R * steps / dt, 1), "unit": "points/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 3), "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "dtype": "ristretto255 / fq252",
        "data": "synthetic scalars (splitmix64 seed 7) resident in HBM, generators MultiCommitGens(1024, spg_bench_rows)",
        "config": {"workload": "row-batch MSM, SURVEY 8d config 2 (1024 row-MSMs x 1024)", "rows": L, "width": R},
        "roofline": roof, "roofline_hbm": roof_h, "roofline_valu": roof_v,
        "valu_whole_commit": {"madds_per_commit": madds, "device_us_per_commit": round(dev_us, 1),
                              "madds_per_s": round(madds / (dev_us * 1e-6), 1) if dev_us else None,
                              "frac_of_peak": round(madds / (dev_us * 1e-6) / MADD_PEAK, 4) if dev_us else None},
        "precomputation": pre, "no_table": no_tab,
        "cpu_baseline": cpu, "cpu_baseline_all_cores": cpu_all, "rows_bitexact_vs_cpu": bitexact,
        "rows_sha256": hashlib.sha256(sorted(outs)[0]).hexdigest()[:16], "kernels": kernel_table(prof, steps, top=8),
    }


# ---------------------------------------------------------------- config 1: the CPU path alone
def cpu1_core(log_cons=10, log_proofs=1):
    """SURVEY 8d config 1 (benches/snark.rs: synthetic R1CS of 2^12 constraints, CPU reference path only, plumbing):
    one SNARK::prove of the 2-block x 2^log_proofs x 2^log_cons program by the CPU oracle on 1 host thread, with the
    per-phase wall times under the labels of the reference's Timer scopes (src/timer.rs, src/lib.rs:1088-2692)."""
    import workload

    po = oracle()
    wl = workload.SnarkWorkload(num_blocks=2, log_cons=log_cons, log_proofs=log_proofs, num_vars=1 << log_cons)
    _, rc = po.snark_prove(wl, workload.tape_seed(), gens_label=GENS_LABEL, gens_num_vars=GENS_NUM_VARS,
                           label=b"snark_bench")
    tp = po.snark_last_prove_us() * 1e-6
    N = wl.total_constraints
    return {"metric": "R1CS constraints/sec (SNARK::prove), CPU path only", "value": round(N / tp, 1),
            "unit": "constraints/s", "cores": 1, "kind": "port", "ms_per_prove": round(tp * 1e3, 2),
            "config": {"workload": "SNARK::prove (src/lib.rs:971-2746), SURVEY 8d config 1", "constraints": N,
                       "block_types": 2, "executions_per_block": 1 << log_proofs, "constraints_per_block": 1 << log_cons},
            "oracle_verifier_status": rc,
            "phases_ms": {k: round(us * 1e-3, 3) for k, us in po.snark_last_phases()}}


# ---------------------------------------------------------------- MSM (config 2)
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


def msm_core(env, ctx, log_msm, steps, warmup, cpu_on, traffic_file=None):
    """one 2^k-point MSM (GroupElement::vartime_multiscalar_mul, src/group.rs:98-116) against
    MultiCommitGens::new(2^k, b"spg_bench_msm").G, resident in HBM. With N ranks the MSM is split into contiguous
    chunks: each rank computes an uncompressed partial sum (spg_msm_partial), the 128-byte partials are
    allgathered and added exactly on the host (shard.py) -> strong scaling. A step is one whole MSM ending in the
    32-byte compressed result on every rank."""
    import spg
    import shard

    n = 1 << log_msm
    gens = spg.Gens(ctx, n, b"spg_bench_msm")
    sc = msm_scalars(n)
    # the scalars are resident in HBM before the timed region (uploaded once: spg_msm_buf on one GPU,
    # spg_msm_partial_buf per shard); the host-scalar entry point (spg_msm_partial: its 2^k x 32 B upload inside
    # the call) is timed beside it
    sbuf = spg.Buf(ctx, sc)
    partial = shard.gpu_partial_resident(gens, sbuf)
    partial_host = shard.gpu_partial(gens, sc)

    def run(part):
        if env.dist is None:
            return spg.points_sum_compress([part(0, n)])
        return shard.sharded_msm(env.dist, part, n, env.comm_device if env.backend == "nccl" else None)[0]

    def step():
        if env.dist is None:  # one call: spg_msm_buf (vartime_multiscalar_mul -> 32 compressed bytes)
            return gens.msm_buf(sbuf)
        return run(partial)

    outs_raw = set()

    def step_keep():
        r = step()
        outs_raw.add(r)
        return r

    c0 = spg.comb_stats()
    dt, laps, _ = timed(env, step_keep, steps, warmup)
    pre = precomputation(c0, spg.comb_stats(), "comb table of MultiCommitGens(2^k, spg_bench_msm) (c = 9 windows, "
                                               "128-byte entries), built in the first (warmup) step and kept in HBM; the "
                                               "CPU baseline is the table-free vartime Pippenger")
    no_tab = no_table_leg(env, ctx, step, steps, warmup, outs_raw)

    def step_host():
        r = run(partial_host)
        outs_raw.add(r)
        return r

    dt_host, _, _ = timed(env, step_host, steps, warmup)
    assert len(outs_raw) == 1, "MSM result changed between steps (or between the two entry points)"
    prof = profile_pass(ctx, step, steps)
    roof, roof_h, roof_v = rooflines(prof, traffic_file)
    lo, hi = shard.chunk(n, env.rank, env.world)
    dev_us = prof.busy_us / steps
    madds = sum(v[3] for v in prof.values()) / steps
    cpu = cpu_all = bitexact = None
    if env.rank == 0 and cpu_on:
        import numpy as np

        po = oracle()
        pts = gens.compressed()
        ref_pts = po.gens_stream(b"spg_bench_msm", n + 1)
        tc = time.perf_counter()
        ref = po.msm(ref_pts[:n], sc)
        tcpu = time.perf_counter() - tc
        bitexact = bool(np.array_equal(pts, ref_pts) and ref in outs_raw)
        if env.world == 1:
            cpu = {"value": round(n / tcpu, 1), "unit": "points/s", "cores": 1, "kind": "port",
                   "sample": f"the whole MSM ({n} pairs) by the oracle's vartime Pippenger restatement incl. point "
                             f"decompression, {tcpu:.2f} s on 1 host thread"}
            cpu_all = all_cores_baseline(lambda: po.msm(ref_pts[:n], sc), n, "points/s",
                                         f"the whole {n}-point MSM by the oracle's vartime Pippenger")
    return {
        "metric": "MSM points/sec (GroupElement::vartime_multiscalar_mul, 2^%d points); result bit-exact" % log_msm,
        "value": round(n * steps / dt, 1), "unit": "points/s", "n_gpus": env.world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(dt / steps * 1e3, 3),
        "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3), "higher_is_better": True,
        "ms_per_step_incl_scalar_upload": round(dt_host / steps * 1e3, 3),
        "scaling": "strong", "dtype": "ristretto255 / fq252",
        "data": "synthetic scalars (splitmix64 seed 1 + edge cases) resident in HBM, generators "
                "MultiCommitGens(2^k, spg_bench_msm)",
        "config": {"workload": "single MSM, SURVEY 8d config 2", "points": n,
                   "parallelism": f"contiguous shards x{env.world}, allgather of partials ({env.backend})"},
        "roofline": roof, "roofline_hbm": roof_h, "roofline_valu": roof_v,
        # the whole launch sequence of one MSM: madds over all its kernels' time (points/s is the metric)
        "valu_whole_msm": {"madds_per_msm": madds, "device_us_per_msm": round(dev_us, 1),
                           "madds_per_s": round(madds / (dev_us * 1e-6), 1) if dev_us else None,
                           "frac_of_peak": round(madds / (dev_us * 1e-6) / MADD_PEAK, 4) if dev_us else None},
        "precomputation": pre, "no_table": no_tab,
        "cpu_baseline": cpu, "cpu_baseline_all_cores": cpu_all, "result_bitexact_vs_cpu": bitexact,
        "result": sorted(outs_raw)[0].hex(), "kernels": kernel_table(prof, steps, top=12),
    }


def main_msm(a):
    env = Env(a)
    import spg

    ctx = spg.Context(env.gpu)
    out = msm_core(env, ctx, a.log_msm, a.steps, a.warmup, not a.no_cpu_baseline,
                   a.traffic or (TRAFFIC["msm16"] if a.log_msm == 16 else None))
    if env.rank == 0:
        out["vs_baseline"] = None
        print(json.dumps(out))
    env.close()


# ---------------------------------------------------------------- SPARK (config 5)
def spark_core(env, ctx, k, cpu_log_nnz, steps, warmup, mode, cpu_on, traffic_file=None, comm="auto"):
    """SparseMatPolynomial::multi_evaluate + SparseMatPolyEvalProof::prove over the three
    2^k-nonzero matrices (A, B, C) with num_vars_x = num_vars_y = k. A step is one multi_evaluate at (rx, ry)
    plus one full SPARK evaluation proof (derefs, derefs commit, hash layer, product trees, batched layer
    sumchecks, hash-layer PolyEvalProofs) with the dense representation resident in HBM (multi_commit is the
    preprocessing step, SNARK::encode, and is timed separately). Multi-GPU (mode shard): ONE proof split over the
    ranks (spg_set_comm; SURVEY 8e: Hyrax rows, interleaved product trees, per-round (e0, e2, e3) allgathers)
    -> strong scaling; mode replicas: an independent proof per rank (weak)."""
    import numpy as np

    import spg
    import workload

    shard = env.world > 1 and mode == "shard"
    transport = install_comm(env, ctx, comm) if shard else None
    t0 = time.perf_counter()
    wl = workload.SparkWorkload(k)
    views = workload.CViews(wl)
    t_gen = time.perf_counter() - t0
    rng = np.random.default_rng(3 + (0 if shard else env.rank))
    r = rng.integers(0, 1 << 63, size=(2 * k, 4), dtype=np.uint64)
    r[:, 3] &= np.uint64((1 << 60) - 1)
    rx, ry = r[:k], r[k:]
    c0 = spg.comb_stats()
    t0 = time.perf_counter()
    comm = spg.SparkCommitment(ctx, views.inst, b"gens_r1cs_eval", wl.nnz, 3)
    t_commit = time.perf_counter() - t0
    inst = spg.R1CSInst(ctx, views.inst)
    seed = workload.tape_seed()

    def step():
        evals = spg.r1cs_multi_evaluate(ctx, inst, 1, rx, ry)
        return comm.prove(rx, ry, evals, spg.Transcript(b"spark_bench"), spg.RandomTape(b"proof", seed))

    dt, laps, proofs = timed(env, step, steps, warmup)
    pre = precomputation(c0, spg.comb_stats(), "comb tables of the gens_r1cs_eval generator sets (comb_ops / comb_mem "
                                               "rows at the commitment, the derefs rows in the first proof), kept in HBM; "
                                               "the CPU baseline uses no tables")
    prof = profile_pass(ctx, step, steps)
    same = None
    if shard:  # every rank of one sharded proof must hold the same bytes, the same in every step
        hs = [None] * env.world
        env.dist.all_gather_object(hs, sorted(proofs))
        same = all(h == hs[0] for h in hs) and len(hs[0]) == 1
        ctx.set_comm(0, 1)
    else:
        assert len(proofs) == 1, "proof bytes changed between steps"
    nnz = 3 * wl.nnz
    value = nnz * (1 if shard else env.world) * steps / dt
    roof, roof_h, roof_v = rooflines(prof, traffic_file)
    cpu = cpu_all = None
    if env.rank == 0 and env.world == 1 and cpu_on:
        po = oracle()
        kc = min(cpu_log_nnz, k)
        wc = workload.SparkWorkload(kc)
        rc_ = rng.integers(0, 1 << 63, size=(2 * kc, 4), dtype=np.uint64)
        rc_[:, 3] &= np.uint64((1 << 60) - 1)
        po.spark_prove(wc, rc_[:kc], rc_[kc:], seed)
        tcpu = po.spark_last_prove_us() * 1e-6
        sample = (f"3 x 2^{kc} nonzeros (same generator; the GPU line proves 3 x 2^{k}), multi_evaluate + "
                  f"SparseMatPolyEvalProof::prove")
        cpu = {"value": round(3 * (1 << kc) / tcpu, 1), "unit": "nonzeros/s", "cores": 1, "kind": "port",
               "sample": f"{sample}, {tcpu:.2f} s on 1 host thread (the commitment is preprocessing, untimed)"}
        # all cores: one oracle copy per usable core commits, all meet at a barrier, then all prove at once; the wall
        # time runs from the first prove's start to the last one's end (verification skipped)
        k_all = usable_cores()
        dt_all = po.spark_concurrent_prove(wc, rc_[:kc], rc_[kc:], seed, k_all)
        cpu_all = {"value": round(3 * (1 << kc) * k_all / dt_all, 1), "unit": "nonzeros/s", "cores": k_all,
                   "kind": "port",
                   "sample": f"{k_all} concurrent independent copies of: {sample}, proving together after a barrier; "
                             f"{dt_all:.2f} s wall from the first prove's start to the last one's end"}
    return {
        "metric": "SPARK nonzeros/sec (sparse_mlpoly multi_evaluate + SparseMatPolyEvalProof::prove)",
        "value": round(value, 1), "unit": "nonzeros/s", "n_gpus": env.world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 3), "ms_per_step_median": round(sorted(laps)[len(laps) // 2] * 1e3, 3),
        "higher_is_better": True, "scaling": "strong" if shard else "weak",
        "dtype": "fq252 (8x u32 Montgomery limbs), ristretto255", "data": "synthetic (SURVEY 8d config 5 generator, seed 5)",
        "config": {"workload": "SparseMatPolyEvalProof::prove, batch 3 (src/sparse_mlpoly.rs:1497-1564)",
                   "log_nnz": k, "num_vars_x": k, "num_vars_y": k,
                   "parallelism": f"one proof sharded x{env.world} ({transport})" if shard else f"replicas x{env.world}"},
        "roofline": roof, "roofline_hbm": roof_h, "roofline_valu": roof_v,
        "roofline_fq": roofline_fq(prof, traffic_file), "cpu_baseline": cpu,
        "cpu_baseline_all_cores": cpu_all, "proof_sha256": sorted(proofs)[0][:16], "ranks_agree": same,
        "transport": transport,
        "commit_s": round(t_commit, 3), "host_gen_s": round(t_gen, 3), "precomputation": pre,
        "device_busy_ms_per_step": round(prof.busy_us / steps / 1e3, 3),
        "kernels": kernel_table(prof, steps),
    }


def main_spark(a):
    env = Env(a)
    import spg

    ctx = spg.Context(env.gpu)
    out = spark_core(env, ctx, a.log_nnz, a.cpu_log_nnz, a.steps, a.warmup, a.mode or "shard", not a.no_cpu_baseline,
                     a.traffic or (TRAFFIC["spark24"] if a.log_nnz == 24 else None), a.comm)
    if env.rank == 0:
        out["vs_baseline"] = None
        print(json.dumps(out))
    env.close()


def main_rows(a):
    env = Env(a)
    import spg

    ctx = spg.Context(env.gpu)
    out = rows_core(env, ctx, a.steps, a.warmup, not a.no_cpu_baseline, a.traffic or TRAFFIC["rows"])
    if env.rank == 0:
        out["vs_baseline"] = None
        print(json.dumps(out))
    env.close()


def main_launchcheck(a):
    """the launcher's own check (tests/test_bench_launch.py, CPU): every rank joins the process group and rank 0
    prints the world it saw and the sum of the ranks -- no libspg, no GPU"""
    env = Env(a)
    s = env.world * (env.world - 1) // 2
    if env.dist is not None:
        t = env.torch.tensor([float(env.rank)])
        env.dist.all_reduce(t)
        s = int(t.item())
    if env.rank == 0:
        print(json.dumps({"n_gpus": env.world, "rank_sum": s, "launcher": os.environ.get("SPG_BENCH_LAUNCHER")}))
    env.close()


# ---------------------------------------------------------------- N ranks without torchrun
def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_envs(n, base, port):
    """the torch.distributed env:// variables of n local ranks (one per GPU: LOCAL_RANK r drives GPU r)"""
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 ROLE_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPG_BENCH_LAUNCHER="bench.py")
        out.append(e)
    return out


def check_world(gpus, environ):
    """a rank started by torchrun (WORLD_SIZE set) must be one of --gpus ranks: returns an error string or None"""
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return None
    if not ws.isdigit() or int(ws) != gpus:
        return f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}; launch --gpus N under torchrun with --nproc-per-node N"
    return None


def launch(gpus, argv):
    """`bench.py --gpus N` with N > 1 and no torchrun: start N child ranks of this same command (one per GPU,
    env:// rendezvous on 127.0.0.1) before anything here touches a GPU; rank 0's stdout is the line, the others'
    goes to stderr. Returns the exit code: the first failing rank's, after the others are stopped."""
    import signal
    import subprocess

    port = free_port()
    procs = []
    for r, e in enumerate(child_envs(gpus, os.environ, port)):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e,
                                      stdout=None if r == 0 else sys.stderr.fileno()))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, lambda *x: (stop(), sys.exit(143)))
    rc = 0
    while procs and any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            stop()
            break
        time.sleep(0.05)
    for p in procs:
        p.wait()
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    return rc


def main():
    a = parse()
    err = check_world(a.gpus, os.environ)
    if err:
        print(err, file=sys.stderr)
        sys.exit(2)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(a.gpus, sys.argv[1:]))
    {"snark": main_snark, "r1cs": main_r1cs, "spark": main_spark, "msm": main_msm, "rows": main_rows,
     "launchcheck": main_launchcheck}[a.workload](a)


if __name__ == "__main__":
    main()
