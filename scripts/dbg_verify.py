import sys, os
sys.path[:0]=['spartan-parallel_amd','tests']
os.environ["SPG_DEBUG_TR"]="1"
import spg, workload
from r1cs_cases import SNARK_CASES
ctx = spg.Context(0)
g = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1<<24)
wl = workload.SnarkWorkload(**SNARK_CASES["b2_x32_q2"])
v = workload.SnarkViews(wl)
b, p, r = spg.SnarkComp(ctx, v.block, multi=True), spg.SnarkComp(ctx, v.pairwise), spg.SnarkComp(ctx, v.perm_root)
w = spg.SnarkWitness(ctx, v.inputs)
pf = spg.snark_prove(ctx, b, p, r, w, g, spg.Transcript(b"snark_test"), spg.RandomTape(b"proof", workload.tape_seed()))
print("proved", len(pf), flush=True)
print(spg.snark_verify(ctx, b, p, r, v.inputs, g, spg.Transcript(b"snark_test"), pf), flush=True)
