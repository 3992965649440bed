#!/bin/bash
# triple layer rounds: kernel phases against the pair, parity of every layer form, then an ABBA A/B of the prove
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
(cd scripts/micro && TRIPLE_ONLY=1 timeout -k 10 120 ./layer_phases > ../../gpurun_out/triple_phases.txt 2>&1) || { cat gpurun_out/triple_phases.txt; exit 1; }
grep -v armed gpurun_out/triple_phases.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  "tests/test_gpu_spark.py" "tests/test_gpu_snark.py::test_round_forms" -k "spark or layer" > gpurun_out/t22.log 2>&1
rc=$?; tail -3 gpurun_out/t22.log; [ $rc = 0 ] || exit $rc
bash scripts/ab_env2.sh SPG_LAYER_TRIPLE 0 1 3 > gpurun_out/ab22_triple.txt
cat gpurun_out/ab22_triple.txt
