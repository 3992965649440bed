#!/bin/bash
# 2-rank gloo rehearsal of the multi-GPU bench line on the final tree (both ranks on the one GPU)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29545 \
  bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --extras r1cs,spark > gpurun_out/b45_2ranks.json 2> gpurun_out/b45_2ranks.err \
  || { tail -20 gpurun_out/b45_2ranks.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b45_2ranks.json").read().strip().splitlines()[-1])
print(d["metric"], d["value"], d["n_gpus"], d["ms_per_step"])
for k in ("config4_r1cs", "config5_spark"):
    c = d.get(k) or {}
    print(k, c.get("ms_per_step"), c.get("ranks_agree"), c.get("transport"), c.get("proof_sha256"))
PY
