import sys, os
sys.path[:0] = ['spartan-parallel_amd', 'oracle', 'tests']
import workload, spg
ctx = spg.Context(0)
g = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
w = workload.SnarkWorkload(num_blocks=2, log_cons=5, log_proofs=1, num_vars=32)
v = workload.SnarkViews(w)
b = spg.SnarkComp(ctx, v.block, multi=True); p = spg.SnarkComp(ctx, v.pairwise); pr = spg.SnarkComp(ctx, v.perm_root)
wit = spg.SnarkWitness(ctx, v.inputs)
pf = spg.snark_prove(ctx, b, p, pr, wit, g, spg.Transcript(b"snark_test"), spg.RandomTape(b"proof", workload.tape_seed()))
print(len(pf))
