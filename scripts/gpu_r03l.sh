#!/bin/bash
# Round 3: wall-clock samples of SNARK::prove's calling thread (scripts/host_sample.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SPG_LIB=$R/spartan-parallel_amd/lib/libspg_fp.so timeout -k 10 300 python scripts/host_sample.py 20 > gpurun_out/host_sample.out 2> gpurun_out/host_sample.err
rc=$?; cat gpurun_out/host_sample.out; tail -3 gpurun_out/host_sample.err; exit $rc
