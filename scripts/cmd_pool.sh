# segment sums of the batch MSM: quad form for the 1024-row block_vars commit (SPG_SEG_QUAD_MAX) A/B
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 16384 1048576; do
    SPG_SEG_QUAD_MAX=$v timeout -k 5 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_ab.json 2>/dev/null || exit $?
    echo "seg_quad_max=$v $(python -c 'import json;d=json.load(open("gpurun_out/b_ab.json"));k=d["kernels"];print(d["ms_per_step"], d.get("ms_per_step_median"), d.get("ms_per_step_min"), {n: v["ms_per_step"] for n, v in k.items() if "msm" in n})')"
  done
done
