"""Per-kernel duration and the idle gap before each launch (previous kernel's end -> this kernel's start on the
device), from a rocprofv3 --kernel-trace CSV: where a transcript-sequential round's wall time goes besides the kernel.
kernel_gaps.py DIR [name-substring ...]  (DIR searched for *kernel_trace.csv; only the main queue's kernels count)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, pats):
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in fs:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # MARK=substring [SKIP=k]: keep the window from the (k+1)-th launch of the marker kernel (the first of each prove)
    # to the end, and report per-prove figures (the warm-up prove and the setup before it left out)
    mark = os.environ.get("MARK")
    nprove = 1
    if mark:
        ix = [i for i, r in enumerate(rows) if mark in r[2]]
        skip = int(os.environ.get("SKIP", "1"))
        if len(ix) > skip:
            rows = rows[ix[skip]:]
            nprove = len(ix) - skip
        print(f"window: {nprove} proves from launch {skip} of {mark!r}; wall {(rows[-1][1] - rows[0][0]) / 1e6 / nprove:.2f} "
              f"ms per prove")
    acc = defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # launches, duration ns, gap ns, max gap
    prev_end = None
    for s, e, n in rows:
        key = n.split("(")[0].replace("void ", "")[:60]
        if prev_end is not None and (not pats or any(p in key for p in pats)):
            g = max(0, s - prev_end)
            a = acc[key]
            a[0] += 1
            a[1] += e - s
            a[2] += g
            a[3] = max(a[3], g)
        prev_end = max(prev_end or 0, e)
    for k, (n, du, ga, mx) in sorted(acc.items(), key=lambda kv: -kv[1][1] - kv[1][2])[:25]:
        print(f"{k:62s} n={n:6d} dur={du / n / 1e3:7.2f} us gap_before={ga / n / 1e3:7.2f} us (total dur "
              f"{du / 1e6:7.2f} ms, gaps {ga / 1e6:7.2f} ms)")
    # idle device time by the (previous kernel -> next kernel) transition: where the host holds the device up
    tr = defaultdict(lambda: [0, 0.0])
    prev = None
    busy_end = None
    for s, e, n in rows:
        key = n.split("(")[0].replace("void ", "").replace("spg::", "")[:34]
        if prev is not None and busy_end is not None and s > busy_end:
            t = tr[(prev, key)]
            t[0] += 1
            t[1] += s - busy_end
        prev = key
        busy_end = max(busy_end or 0, e)
    tot = sum(v[1] for v in tr.values())
    busy = sum(e - s for s, e, _ in rows)
    print(f"-- idle gaps by transition, per prove (idle {tot / 1e6 / nprove:.2f} ms, kernel time {busy / 1e6 / nprove:.2f} ms):")
    for (a, b), (n, g) in sorted(tr.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"  {a:34s} -> {b:34s} n={n / nprove:7.1f} avg {g / n / 1e3:7.2f} us total {g / 1e6 / nprove:6.3f} ms")


def events_in_gaps(d, evfile, top=40):
    """the largest idle gaps of the device in the MARK window, each with the host laps (SPG_TRACE_EVENTS lines of
    evfile: [spgev] <ns> <title>:<lap> <us>) that ended inside it: which host phase held the device up"""
    fs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in fs:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]))
    rows.sort()
    ev = []
    for line in open(evfile):
        if line.startswith("[spgev]"):
            f = line.split()  # lap titles may hold spaces
            ev.append((int(f[1]), " ".join(f[2:-1]), float(f[-1])))
    ev.sort()
    mark = os.environ.get("MARK")
    if mark:
        ix = [i for i, r in enumerate(rows) if mark in r[2]]
        skip = int(os.environ.get("SKIP", "1"))
        rows = rows[ix[skip]:]
    gaps = []
    end = rows[0][1]
    for i in range(1, len(rows)):
        s, e, n = rows[i]
        if s > end:
            gaps.append((s - end, end, s, rows[i - 1][2], n))
        end = max(end, e)
    import bisect
    keys = [x[0] for x in ev]
    by_lap = defaultdict(float)
    maxlap = max((x[2] for x in ev), default=0) * 1e3
    only = os.environ.get("TRANS")  # "prev->next": only the gaps of that kernel transition
    if only:
        pa, pb = [x.strip() for x in only.split("->")]
        gaps = [x for x in gaps if pa in x[3] and pb in x[4]]
    for g, a, b, pn, nn in gaps:
        # every lap whose interval [end - us, end] overlaps the gap, by the overlap (nested Laps objects overlap each
        # other: read the innermost names)
        lo, hi = bisect.bisect_left(keys, a), bisect.bisect_right(keys, b + maxlap)
        for j in range(lo, hi):
            e1 = ev[j][0]
            e0 = e1 - ev[j][2] * 1e3
            ov = min(e1, b) - max(e0, a)
            if ov > 0:
                by_lap[ev[j][1]] += ov
    if os.environ.get("DUMP"):
        # one prove's timeline: every gap over DUMP us between the first two MARK launches, with the laps that
        # overlap it (start offset in the gap, us)
        lim = float(os.environ["DUMP"]) * 1e3
        m2 = [r for r in rows if mark and mark in r[2]]
        stop = m2[1][0] if len(m2) > 1 else rows[-1][1]
        t0 = rows[0][0]
        for g, a, b, pn, nn in gaps:
            if b > stop:
                break
            if g < lim:
                continue
            lo, hi = bisect.bisect_left(keys, a), bisect.bisect_right(keys, b + maxlap)
            laps = []
            for j in range(lo, hi):
                e1 = ev[j][0]
                e0 = e1 - ev[j][2] * 1e3
                if min(e1, b) - max(e0, a) > 0 and ev[j][2] * 1e3 < 4 * g:
                    laps.append(f"{ev[j][1].split(':')[-1]}[{(e0 - a) / 1e3:.0f},{ev[j][2]:.0f}]")
            print(f"{(a - t0) / 1e3:9.0f} {g / 1e3:7.1f} us {pn[-24:]:>24s} -> {nn[-24:]:24s} {' '.join(laps)}")
    tot = sum(g[0] for g in gaps)
    print(f"-- idle {tot / 1e6:.2f} ms in {len(gaps)} gaps; host laps ending inside them (lap time, capped at the gap):")
    for k, v in sorted(by_lap.items(), key=lambda kv: -kv[1])[:top]:
        print(f"  {k:60s} {v / 1e6:8.3f} ms")


if __name__ == "__main__":
    if os.environ.get("EVENTS"):
        events_in_gaps(sys.argv[1], os.environ["EVENTS"])
    else:
        main(sys.argv[1], sys.argv[2:])
