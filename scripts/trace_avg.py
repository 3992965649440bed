"""Mean of the SPG_TRACE=1 SNARK::prove breakdowns in a stderr log, skipping the first (warm-up) prove:
trace_avg.py LOG [fields...]"""
import re
import sys

rows = []
for line in open(sys.argv[1]):
    if "SNARK::prove host breakdown" in line:
        rows.append({k: float(v) for k, v in re.findall(r"(\w[\w+]*)=([\d.]+)", line)})
rows = rows[1:]
fields = sys.argv[2:] or ["input_commit", "block_sat", "block_eval", "total"]
print(len(rows), " ".join(f"{f}={sum(r.get(f, 0) for r in rows) / max(1, len(rows)):.0f}" for f in fields))
