#!/bin/bash
# round-5 GPU call: the segfault of `bench.py --extras r1cs,spark` (CPU baselines on) under faulthandler
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
grep -m1 -o "avx512ifma" /proc/cpuinfo || echo "no avx512ifma"
timeout -k 10 600 python -X faulthandler bench.py --steps 10 --warmup 2 --extras r1cs,spark > gpurun_out/b5.json 2> gpurun_out/b5.err
rc=$?
echo "rc=$rc"
grep -v "amdgpu.ids" gpurun_out/b5.err | tail -40
exit $rc
