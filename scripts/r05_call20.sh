#!/bin/bash
# round-5: the driver's default bench command, smoke(), and the 2-rank gloo rehearsal of the N > 1 line on one GPU
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/b20_full.json 2> gpurun_out/b20_full.err || { tail -30 gpurun_out/b20_full.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/b20_full.json || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke20.log 2>&1 || { tail gpurun_out/smoke20.log; exit 1; }
tail -2 gpurun_out/smoke20.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --extras-log-nnz 20 > gpurun_out/b20_2ranks.json 2> gpurun_out/b20_2ranks.err \
  || { tail -30 gpurun_out/b20_2ranks.err; exit 1; }
python3 -c 'import json;d=json.load(open("gpurun_out/b20_2ranks.json"));print("2ranks", d["value"], d["ms_per_step"]);[print(k, (d.get(k) or {}).get("ms_per_step"), (d.get(k) or {}).get("ranks_agree"), (d.get(k) or {}).get("error")) for k in ("config4_r1cs","config5_spark")]'
