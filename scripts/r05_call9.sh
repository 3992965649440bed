#!/bin/bash
# round-5 GPU call: pinned pool burst cost, old vs new pool (micro), library A/B with 5 alternations, kernel trace +
# lap events of the current build
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
(cd scripts/micro && for b in parts_finals_cpu_old parts_finals_cpu parts_finals_cpu_old parts_finals_cpu; do
  timeout -k 10 120 ./$b 176 pin 2>&1 | grep -i "empty" | sed "s/^/$b: /"; done) | tee gpurun_out/pool_pin.txt
timeout -k 10 1000 bash scripts/ab_lib.sh lib/libspg_prev.so lib/libspg.so 5 > gpurun_out/ab_lib9.txt 2>&1 || { cat gpurun_out/ab_lib9.txt; exit 1; }
cat gpurun_out/ab_lib9.txt
bash scripts/session_r05.sh gaps f
