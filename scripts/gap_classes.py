"""Idle device time of one prove by the host phase that held it (kernel_gaps.py DUMP output on stdin): each gap goes to
the first matching class of the laps that overlap it."""
import collections
import re
import sys

tot, cnt = collections.Counter(), collections.Counter()
for line in sys.stdin:
    m = re.match(r"\s*(\d+)\s+([\d.]+) us\s", line)
    if not m:
        continue
    g = float(m.group(2))
    laps = re.findall(r"(\w[\w+]*)\[", line)
    if any(x.startswith("bullet_fold") for x in laps) and "bullet_launch" not in laps:
        k = "host_bullet_proofs"
    elif "bullet_launch" in laps:
        k = "device_bullet_rounds"
    elif "msm_host_final" in laps:
        k = "device_bullet_end"
    elif any(x.startswith(("pair", "round_", "layer")) for x in laps):
        k = "layer_rounds"
    elif any(x.startswith("p1_") for x in laps):
        k = "phase1"
    elif any(x.startswith("p2_") for x in laps):
        k = "phase2"
    elif laps:
        k = "other:" + laps[0]
    else:
        k = "unlabelled"
    tot[k] += g
    cnt[k] += 1
for k, v in tot.most_common(30):
    print(f"{k:40s} {v / 1000:7.3f} ms  n={cnt[k]}")
print(f"{'total':40s} {sum(tot.values()) / 1000:7.3f} ms")
