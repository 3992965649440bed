#!/bin/bash
# round-5 GPU call: parity with the IFMA host sums, A/B of them (SPG_VEC_MIN=0: scalar), and the driver's default
# bench command once (stability of the whole line)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=500 bash scripts/session_r05.sh tests "test_gpu_snark or test_gpu_r1cs or dropin or test_gpu_spark or test_gpu_proto" || exit 1
T=600 bash scripts/session_r05.sh ab SPG_VEC_MIN "0 16" 3 > gpurun_out/ab_vec.txt 2>&1 || { tail gpurun_out/ab_vec.txt; exit 1; }
cat gpurun_out/ab_vec.txt
timeout -k 10 900 python bench.py > gpurun_out/b6_full.json 2> gpurun_out/b6_full.err
rc=$?
echo "bench rc=$rc"
grep -v "amdgpu.ids" gpurun_out/b6_full.err | tail -30
exit $rc
