#!/bin/bash
# HBM fetch per k_bullet_comb launch in the phase micro (back-to-back launches, warm L2) against the prover's average:
# rocprofv3 --pmc FETCH_SIZE of scripts/micro/bullet_comb_phases, grouped by grid size
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/bc_pmc" -o f -- "$R/scripts/micro/bullet_comb_phases" > "$R/gpurun_out/bc_pmc.out" 2>&1) || { tail -5 gpurun_out/bc_pmc.out; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/bc_pmc/**/*counter_collection.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
acc = collections.defaultdict(list)
for r in rows:
    if "bullet_comb" in r["Kernel_Name"] and r["Counter_Name"].startswith("FETCH_SIZE"):
        acc[int(r["Grid_Size"])].append(float(r["Counter_Value"]))
out = open("gpurun_out/bc_pmc_summary.txt", "w")
for g in sorted(acc):
    v = acc[g]
    line = "grid %7d threads: %3d launches, FETCH_SIZE mean %.1f KiB (x2 gfx950: %.0f bytes per launch), min %.1f max %.1f" % (
        g, len(v), sum(v) / len(v), 2048 * sum(v) / len(v), min(v), max(v))
    print(line); out.write(line + "\n")
PY
