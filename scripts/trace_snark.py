"""SPG_TRACE=1 host-time breakdown of SNARK::prove at the bench shape (prints from libspg on stderr)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "spartan-parallel_amd")]
import spg  # noqa: E402
import workload  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 9
ctx = spg.Context(0)
g = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
w = workload.SnarkWorkload(num_blocks=2, log_cons=10, log_proofs=k, num_vars=1024)
v = workload.SnarkViews(w)
b, p, pr = spg.SnarkComp(ctx, v.block, multi=True), spg.SnarkComp(ctx, v.pairwise), spg.SnarkComp(ctx, v.perm_root)
wit = spg.SnarkWitness(ctx, v.inputs)
for i in range(int(os.environ.get("TRACE_REPS", "3"))):
    spg.snark_prove(ctx, b, p, pr, wit, g, spg.Transcript(b"t"), spg.RandomTape(b"proof", workload.tape_seed()))
