#!/bin/bash
# which phase differs between SPG_HALVED_ENC=0 and 1 (SPG_TRACE=2 breakdowns, 8 proves each, twice)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for v in 0 1 1 0; do
  SPG_HALVED_ENC=$v SPG_TRACE=2 timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --extras none \
    > gpurun_out/b29_$v.json 2> gpurun_out/b29_$v.err || { tail -20 gpurun_out/b29_$v.err; exit 1; }
  python3 - gpurun_out/b29_$v.err $v gpurun_out/b29_$v.json <<'PY'
import sys, re, json, collections
acc = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.search(r"\[spg\] (.*) host breakdown \(us\): (.*)", line)
    if not m: continue
    for kv in m.group(2).split():
        k, v = kv.split("=")
        acc[(m.group(1), k)].append(float(v))
d = json.load(open(sys.argv[3]))
print("HALVED", sys.argv[2], "ms", d["ms_per_step"], "median", d.get("ms_per_step_median"), "dev", d.get("device_busy_ms_per_step"))
for (t, k), v in sorted(acc.items()):
    if t in ("SNARK::prove", "commit queue flush") or k == "total":
        v = v[-8:]
        print("  %-45s %-22s %8.0f" % (t[:45], k, sum(v) / len(v)))
PY
done
