"""Where the calling thread of SNARK::prove spends its wall time (scripts/micro/sampler.c: a per-thread POSIX timer
samples the instruction pointer every 20 us). Writes gpurun_out/host_samples.json: per module, the sampled offsets
(symbolise libspg.so offsets with addr2line / nm here). Not part of the product."""
import collections
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "spartan-parallel_amd")]
import numpy as np  # noqa: E402

import spg  # noqa: E402
import workload  # noqa: E402

ctx = spg.Context(0)
g = spg.R1CSGens(ctx, b"gens_r1cs_sat", 1 << 24)
w = workload.SnarkWorkload(num_blocks=2, log_cons=10, log_proofs=9, num_vars=1024)
v = workload.SnarkViews(w)
b, p, pr = spg.SnarkComp(ctx, v.block, multi=True), spg.SnarkComp(ctx, v.pairwise), spg.SnarkComp(ctx, v.perm_root)
wit = spg.SnarkWitness(ctx, v.inputs)
for _ in range(3):
    spg.snark_prove(ctx, b, p, pr, wit, g, spg.Transcript(b"t"), spg.RandomTape(b"proof", workload.tape_seed()))
S = ctypes.CDLL(os.path.join(ROOT, "scripts", "micro", "libsampler.so"))
S.sampler_start.argtypes = [ctypes.c_size_t, ctypes.c_long]
S.sampler_stop.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
S.sampler_stop.restype = ctypes.c_size_t
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cap = 1 << 24
assert S.sampler_start(cap, 20000) == 0
import time  # noqa: E402

t0 = time.perf_counter()
for _ in range(steps):
    spg.snark_prove(ctx, b, p, pr, wit, g, spg.Transcript(b"t"), spg.RandomTape(b"proof", workload.tape_seed()))
dt = time.perf_counter() - t0
out = np.zeros(cap, dtype=np.uint64)
k = S.sampler_stop(out.ctypes.data, cap)
maps = []
for line in open("/proc/self/maps"):
    f = line.split()
    if len(f) >= 6 and "x" in f[1]:
        lo, hi = (int(x, 16) for x in f[0].split("-"))
        maps.append((lo, hi, int(f[2], 16), f[5]))
def where(a):
    for lo, hi, off, path in maps:
        if lo <= a < hi:
            return (os.path.basename(path), a - lo + off)
    return ("?", 0)


REC = 64  # words per sample: RIP, 3 frame-pointer callers, 60 stack words
spg_maps = [(lo, hi) for lo, hi, off, path in maps if "libspg" in os.path.basename(path)]
cnt = collections.Counter()
stacks = collections.Counter()
flat = out[:k].tolist()
for i in range(0, len(flat) - REC + 1, REC):
    rec = flat[i:i + REC]
    frames = [where(a) for a in rec[:4] if a]
    # first libspg return address on the stack (a caller the frame-pointer chain may miss)
    scan = next((where(a) for a in rec[4:] if any(lo <= a < hi for lo, hi in spg_maps)), ("?", 0))
    frames = tuple(frames) + (scan,)
    cnt[frames[0]] += 1
    stacks[frames] += 1
res = {"steps": steps, "seconds": dt, "samples": int(k) // REC, "period_us": 20,
       "hits": [[m, o, c] for (m, o), c in cnt.most_common()],
       "stacks": [[[list(f) for f in fr], c] for fr, c in stacks.most_common(5000)]}
mods = collections.Counter()
for (m, _), c in cnt.items():
    mods[m] += c
res["by_module"] = dict(mods.most_common())
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "host_samples.json"), "w"))
print(json.dumps({"ms_per_prove": dt / steps * 1e3, "samples": int(k) // REC, "by_module": res["by_module"]}))
