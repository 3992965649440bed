"""Where a headline step's time goes outside the prove's own laps: per call, the Python wrapper's wall time against the
library call's (SPG_TRACE=1 prints `spg_snark_prove call: N us` and the laps' total), for consecutive proves at the
bench shape. Usage: SPG_TRACE=1 python scripts/prove_tail_probe.py 2> gpurun_out/tail.err"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "spartan-parallel_amd")]
import spg  # noqa: E402
import workload  # noqa: E402

ctx = spg.Context(0)
g = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
w = workload.SnarkWorkload(num_blocks=2, log_cons=10, log_proofs=9, num_vars=1024, seed=0x5350415254414E31)
v = workload.SnarkViews(w)
b, p, pr = spg.SnarkComp(ctx, v.block, multi=True), spg.SnarkComp(ctx, v.pairwise), spg.SnarkComp(ctx, v.perm_root)
wit = spg.SnarkWitness(ctx, v.inputs)
seed = workload.tape_seed()
for i in range(int(os.environ.get("TRACE_REPS", "8"))):
    t0 = time.perf_counter()
    proof = spg.snark_prove(ctx, b, p, pr, wit, g, spg.Transcript(b"snark_bench"), spg.RandomTape(b"proof", seed))
    t1 = time.perf_counter()
    print(f"[probe] wrapper call {1e6 * (t1 - t0):.0f} us, proof {len(proof)} bytes", file=sys.stderr, flush=True)
