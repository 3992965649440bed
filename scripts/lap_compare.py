"""Per-proof DotProductProofLog laps (SPG_TRACE=3 stderr lines) averaged by (path, n): lap_compare.py FILE... [LAP]"""
import re,sys,collections
LAP = sys.argv[-1] if not sys.argv[-1].endswith(".err") else "bullet_host"
for f in [a for a in sys.argv[1:] if a.endswith(".err")]:
    acc=collections.defaultdict(list)
    for line in open(f):
        m=re.search(r"DotProductProofLog n=(\d+) (\S+):(.*)",line)
        if not m: continue
        d=dict(kv.split("=") for kv in m.group(3).split())
        acc[(m.group(2),int(m.group(1)))].append((float(d.get(LAP,0)),float(d.get("total",0))))
    for k in sorted(acc):
        v=acc[k]; print(f, k, len(v), LAP + " %.1f"%(sum(a for a,_ in v)/len(v)), "total %.1f"%(sum(b for _,b in v)/len(v)))
