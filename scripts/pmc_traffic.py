#!/usr/bin/env python3
"""Per-launch HBM traffic of the libspg kernels from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section)
FETCH_SIZE on gfx950 reports half the bytes of wide coalesced reads, so reads are doubled; WRITE_SIZE is
taken as is. Both counters count Infinity-Cache hits as traffic (upper bound on HBM bytes).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# device kernel symbol -> libspg profiling scope name (spg_prof_read)
NAMES = {
    # fused fold + evaluation instances first (first match wins)
    "k_phase1_eval_q<true>": "sc_phase1_fold_eval", "k_phase1_eval<true>": "sc_phase1_fold_eval",
    "k_phase2_eval_q<true>": "sc_phase2_fold_eval", "k_phase2_eval<true>": "sc_phase2_fold_eval",
    "k_phase1_pair": "sc_phase1_pair", "k_phase2_pair": "sc_phase2_pair", "k_phase1_fold2x": "sc_fold",
    "k_phase2_fold2x": "sc_fold", "k_pqx_bound_q": "sc_fold_q_all",
    "k_bullet_comb": "msm_bullet_round", "k_comb_msm_parts": "msm_comb_parts", "k_comb_accum": "msm_comb",
    "k_layer_persist": "spark_layer_persist",
    "k_phase1_eval": "sc_phase1_eval", "k_phase2_eval": "sc_phase2_eval", "k_pqx_fold": "sc_fold",
    "k_spmv": "spmv_block", "k_z_fill": "z_fill", "k_abc": "eval_table_abc", "k_bound_part": "poly_bound",
    "k_fold_top": "fold_dense", "k_eq_table": "eq_table", "k_cubic_eval": "sc_cubic_eval",
    "k_final": "msm_final", "k_segments": "msm_segments", "k_items": "msm_bucket_items",
    "k_layer_eval": "spark_layer_eval", "k_layer_tiny": "spark_layer_tiny", "k_fold_many": "spark_fold", "k_seg_dot": "spark_evaluate",
    "k_gather": "spark_deref", "k_bound_rows": "spark_bound", "k_dot3": "spark_dotp_eval",
    "k_tree_level": "spark_product_tree", "k_tree_top": "spark_product_tree", "k_hash_ops": "spark_hash_layer",
    "k_layer_pair": "spark_layer_pair", "k_layer_triple": "spark_layer_triple",
    "k_layer_round_q": "spark_layer_round", "k_layer_round": "spark_layer_round", "k_layer_close": "spark_layer_close",
    "k_bullet_round_q": "msm_bullet_round", "k_big_accum": "msm_big_accum", "k_big_digits": "msm_big_sort",
    "k_big_scatter": "msm_big_sort", "k_smsm_bucket_q": "msm_small_bucket", "k_digits_rows": "msm_digits_rows",
    "k_compress_ext": "msm_compress",
}


def scope(kname):
    for k, v in NAMES.items():
        if "<" in k:  # a template instance: "spg::k_x<true>(...)"
            if ("::" + k) in kname:
                return v
            continue
        if k + "(" in kname or kname.endswith(k) or ("::" + k) in kname:
            return v
    return None


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            s = scope(row.get("Kernel_Name", ""))
            if s:
                acc[s].append(float(row["Counter_Value"]))
    return acc


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    out = {"note": "hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (KiB->bytes), gfx950 correction per "
                   "MI355X_MICROARCH.md; averages over every launch of the profiled bench run", "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fa = sum(f) / len(f) * 1024 if f else 0.0
        wa = sum(w) / len(w) * 1024 if w else 0.0
        out["kernels"][k] = {"launches": max(len(f), len(w)), "fetch_bytes_raw": fa, "write_bytes": wa,
                             "hbm_bytes_per_launch": 2 * fa + wa}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
