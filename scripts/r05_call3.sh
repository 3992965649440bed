#!/bin/bash
# round-5 GPU call: host parts-finals micro on the box, Bullet comb points-per-workgroup A/B (SNARK wall), config-5
# A/B of the comb window width and of paired layer rounds (SPG_TRACE host breakdowns)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
(cd scripts/micro && timeout -k 10 120 ./parts_finals_cpu 704 > ../../gpurun_out/pf_704.txt 2>&1 && \
  timeout -k 10 120 ./parts_finals_cpu 176 > ../../gpurun_out/pf_176.txt 2>&1) || exit 1
cat gpurun_out/pf_704.txt gpurun_out/pf_176.txt
T=600 bash scripts/session_r05.sh ab SPG_BCOMB_R "8 1 2" 2 > gpurun_out/ab_bcomb_r.txt 2>&1 || { tail gpurun_out/ab_bcomb_r.txt; exit 1; }
cat gpurun_out/ab_bcomb_r.txt
mkdir -p gpurun_out/c5
for v in 13 12; do
  SPG_COMB_C_BIG=$v SPG_TRACE=1 timeout -k 10 300 python bench.py --workload spark --log-nnz 24 --steps 5 --warmup 1 \
    --no-cpu-baseline > gpurun_out/c5/b_c$v.json 2> gpurun_out/c5/t_c$v.txt || exit 1
  python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d["ms_per_step"], d.get("ms_per_step_median"), d.get("device_busy_ms_per_step"))' gpurun_out/c5/b_c$v.json
done
SPG_LAYER_PAIR=0 SPG_TRACE=1 timeout -k 10 300 python bench.py --workload spark --log-nnz 24 --steps 5 --warmup 1 \
  --no-cpu-baseline > gpurun_out/c5/b_nopair.json 2> gpurun_out/c5/t_nopair.txt || exit 1
python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d["ms_per_step"], d.get("ms_per_step_median"), d.get("device_busy_ms_per_step"))' gpurun_out/c5/b_nopair.json
