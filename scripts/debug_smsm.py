"""Small-MSM path at window widths 8 and 9 against the big path (bounds-checked library via SPG_LIB)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spartan-parallel_amd"))
import spg  # noqa: E402

ctx = spg.Context(0)
g = spg.Gens(ctx, 4100, b"gens_r1cs_sat")
rng = np.random.default_rng(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 130
s = rng.integers(0, 2**63, (n, 4), dtype=np.uint64)
s[:, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
ref = g.commit_rows(np.concatenate([s] * 5), 5, n)[0].tobytes()  # big path (B = 5 > 4)
for c in sys.argv[2:] or ["8", "9"]:
    os.environ["SPG_SMSM_C"] = c
    out = g.msm(s)
    print(f"n={n} c={c} match={out == ref}", flush=True)
