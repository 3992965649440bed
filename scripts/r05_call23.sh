#!/bin/bash
# untraced per-phase host breakdown of SNARK::prove (SPG_TRACE=2) with the triple layer rounds
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_TRACE=2 timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --extras none \
  > gpurun_out/b23.json 2> gpurun_out/b23.err || { tail -20 gpurun_out/b23.err; exit 1; }
grep "SNARK::prove host breakdown\|R1CSProof::prove host\|ProductCircuitEvalProofBatched::prove host\|SparseMatPolyEvalProof::prove host\|pool bursts\|keccak" gpurun_out/b23.err | tail -40
cat gpurun_out/b23.json
