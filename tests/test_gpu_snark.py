"""SNARK::prove on the GPU (libspg.so: spg_snark_encode / spg_snark_witness_new / spg_snark_prove) vs the CPU
oracle: identical bincode(SNARK) under the same transcript label and RandomTape seed. Small cases are pinned by
tests/golden/snark_proofs.json (oracle proofs its verifier accepted); the larger ones run the oracle live."""
import hashlib
import json
import os

import pytest

from r1cs_cases import GPU_SNARK_CASES, SNARK_CASES

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
GENS_LABEL = b"gens_r1cs_sat"
GENS_NV = 1 << 24


@pytest.fixture(scope="module")
def vars_gens(ctx):
    import spg

    return spg.R1CSGens(ctx, GENS_LABEL, GENS_NV)


def gpu_snark(ctx, vars_gens, wl, seed, label=b"snark_test", repeat=1):
    import spg
    import workload

    v = workload.SnarkViews(wl)
    block = spg.SnarkComp(ctx, v.block, multi=True)
    pairwise = spg.SnarkComp(ctx, v.pairwise)
    perm_root = spg.SnarkComp(ctx, v.perm_root)
    wit = spg.SnarkWitness(ctx, v.inputs)
    out = []
    for _ in range(repeat):
        out.append(spg.snark_prove(ctx, block, pairwise, perm_root, wit, vars_gens, spg.Transcript(label),
                                   spg.RandomTape(b"proof", seed)))
    return out


def _check(got, ref):
    if got != ref:
        from proof_layout import first_diff_snark

        where = first_diff_snark(got, ref) if len(got) == len(ref) else f"length {len(got)} vs {len(ref)}"
        pytest.fail(f"SNARK bytes differ first at {where}")


@pytest.mark.parametrize("case", sorted(SNARK_CASES))
def test_snark_matches_golden(ctx, oracle, vars_gens, case):
    import workload

    wl = workload.SnarkWorkload(**SNARK_CASES[case])
    (proof,) = gpu_snark(ctx, vars_gens, wl, workload.tape_seed())
    golden = json.load(open(os.path.join(G, "snark_proofs.json")))[case]
    if hashlib.sha256(proof).hexdigest() != golden["proof_sha256"]:
        ref, rc = oracle.snark_prove(wl, workload.tape_seed())
        assert rc == 0
        _check(proof, ref)


@pytest.mark.parametrize("case", sorted(GPU_SNARK_CASES))
def test_snark_matches_oracle_large(ctx, oracle, vars_gens, case):
    import workload

    wl = workload.SnarkWorkload(**GPU_SNARK_CASES[case])
    a, b = gpu_snark(ctx, vars_gens, wl, workload.tape_seed(), repeat=2)
    assert a == b, "proof not repeatable"
    ref, rc = oracle.snark_prove(wl, workload.tape_seed())
    assert rc == 0
    _check(a, ref)


@pytest.mark.parametrize("case", ["mem_uneven_b3_x64", "widths_b3_x64"])
def test_circ_program_on_gpu(ctx, vars_gens, tmp_path, case):
    """a program read back from CirC's .ctk/.rtk files (circ.CircProgram, examples/interface.rs) proves on the GPU
    to the golden bytes of the program it was exported from"""
    import circ
    import workload

    ctk, rtk = circ.export_workload(workload.SnarkWorkload(**SNARK_CASES[case]))
    cp, rp = tmp_path / "p_bin.ctk", tmp_path / "p_bin.rtk"
    cp.write_bytes(ctk.to_bytes())
    rp.write_bytes(rtk.to_bytes())
    proof = circ.prove(ctx, circ.CircProgram.load(str(cp), str(rp)), label=b"snark_test", vars_gens=vars_gens)
    golden = json.load(open(os.path.join(G, "snark_proofs.json")))[case]
    assert hashlib.sha256(proof).hexdigest() == golden["proof_sha256"]


ROUND_FORMS = {
    "eval_one_thread": {"SPG_SC_QUAD_MAX": "0"},
    "eval_quad_everywhere": {"SPG_SC_QUAD_MAX": str(1 << 40)},
    "fold_launches": {"SPG_SC_FUSE": "0"},
    "layer_persist": {"SPG_LAYER_PERSIST": "1"},
    "layer_persist_host_polls": {"SPG_LAYER_PERSIST": "1", "SPG_PERSIST_RELAY": "0"},
    "layer_persist_one_wg": {"SPG_LAYER_PERSIST": "1", "SPG_PERSIST_WGS": "1", "SPG_PERSIST_MAX": str(1 << 20)},
    "layer_persist_wide": {"SPG_LAYER_PERSIST": "1", "SPG_PERSIST_WGS": "256", "SPG_PERSIST_MAX": str(1 << 20)},
    "layer_persist_no_ends": {"SPG_LAYER_PERSIST": "1", "SPG_LAYER_ENDS": "0"},
    "z_fill_in_order": {"SPG_Z_SIDE": "0"},
    "z_fill_after_round_0": {"SPG_Z_AFTER": "0"},
    "z_fill_at_phase2": {"SPG_Z_AFTER": "100000"},
    "eq_table_per_launch": {"SPG_EQ_MULTI": "0"},
    "layer_single_rounds": {"SPG_LAYER_PAIR": "0"},
    "layer_pairs_small_wgs": {"SPG_PAIR_BS": "64"},
    # 64-thread pairs asked for up to 6144 elements: the launch plan must cap them at 1536 (the partials workspace)
    "layer_pairs_small_wgs_everywhere": {"SPG_PAIR_BS": "64", "SPG_PAIR_MAX": "6144", "SPG_WIDE_MIN": str(1 << 40),
                                         "SPG_LAYER_TRIPLE": "0"},
    "layer_pairs_everywhere": {"SPG_PAIR_MAX": "6144", "SPG_WIDE_MIN": str(1 << 40)},
    "layer_pairs_no_triples": {"SPG_LAYER_TRIPLE": "0"},
    "layer_triples_everywhere": {"SPG_TRIPLE_MAX": "1536", "SPG_WIDE_MIN": str(1 << 40), "SPG_STEP_COSTS": "18,25,1"},
    "layer_triples_after_pairs": {"SPG_STEP_COSTS": "18,10,12"},
    "witness_parts_copied": {"SPG_WIT_IN_PLACE": "0"},
    "comb_12_bit_windows": {"SPG_COMB_C": "12"},
    "comb_packed_entries": {"SPG_COMB_PAD": "0"},
    "tiny_row_commits_on_host": {"SPG_HOST_COMMIT_MAX": "256"},
    "row_encodings_on_device": {"SPG_HALVED_ENC": "0"},
    "tree_levels_per_launch": {"SPG_TREE_TOP": "0"},
    "tree_one_launch": {"SPG_TREE_TOP": str(1 << 40)},
    "delta_bucket_msm": {"SPG_DELTA_COMB": "0"},
    "bullet_comb_rolled": {"SPG_BCOMB_ROLL": "1"},
    "dotlog_cy_beta_in_order": {"SPG_DOTLOG_EARLY": "0"},
    "delta_scalars_from_host": {"SPG_DELTA_DEV": "0"},
    "spmv_and_z_fill_untiled": {"SPG_SPMV_TILED": "0", "SPG_Z_TILED": "0"},
    "q_folds_one_per_challenge": {"SPG_Q_BOUND_ALL": "0"},
    "opening_combinations_on_calling_thread": {"SPG_AXPY_POOL": "0"},
    "small_commit_jobs_one_slice": {"SPG_ENC_SPLIT": "0"},
    "phase1_single_rounds": {"SPG_P1_PAIR": "0"},
    "phase2_single_rounds": {"SPG_P2_PAIR": "0"},
    "phase2_pairs_small_only": {"SPG_P2_PAIR_MAX": "16"},
    "pairs_up_to_32768_elements": {"SPG_P1_PAIR_MAX": "32768", "SPG_P2_PAIR_MAX": "32768"},
    "phase1_pairs_small_only": {"SPG_P1_PAIR_MAX": "16"},
    "witness_upload_workers": {"SPG_H2D": "1"},
}


@pytest.mark.parametrize("form", sorted(ROUND_FORMS))
def test_round_forms(form):
    """the sumcheck rounds in every launch form, against the golden proof's bytes (the default mixes them by round
    size; a fresh process reads the switches): R1CSProof evaluations one thread per point (SPG_SC_QUAD_MAX=0) or a
    quad per point everywhere; phase-1 and phase-2 folds as launches of their own (SPG_SC_FUSE=0) instead of inside the next
    round's evaluation; SPARK layer rounds in the resident launch (SPG_LAYER_PERSIST=1; the default launches each
    round), with workgroup 0 relaying the host's answer or every workgroup polling the host, with one workgroup over
    every round, with 256 workgroups, and without posting the layer's entries; the R1CS Z fill in stream order
    (SPG_Z_SIDE=0) or on the second stream after phase-1 round 0 or only at phase 2 (SPG_Z_AFTER); one eq table
    per launch (SPG_EQ_MULTI=0); device witness parts copied instead of read in place (SPG_WIT_IN_PLACE=0); SPARK layer
    rounds one per launch (SPG_LAYER_PAIR=0) instead of two per launch where they are small, paired rounds over 64-thread
    workgroups (more of them: the ticketed sums and the last pair's corners from several workgroups), and pairs for every
    round that fits (SPG_PAIR_MAX, no throughput-form rounds); pairs without triples (SPG_LAYER_TRIPLE=0), triples
    wherever they fit (SPG_TRIPLE_MAX, SPG_STEP_COSTS: up to 384 elements, 96 workgroups) and pairs preferred
    before the triples (a triple applying two pending folds); comb tables of 12-bit windows (SPG_COMB_C=12; the default
    is 13 up to 1024 generators) under the row commitments and the Bullet rounds, and comb entries packed at
    96 bytes (SPG_COMB_PAD=0) instead of one 128-byte line each; row commitments of at most 256 scalars on the host pool
    (SPG_HOST_COMMIT_MAX=256) instead of the device; comb row commitments encoded by k_compress_ext
    (SPG_HALVED_ENC=0) instead of from halved points as the host's batched encodings of doubles; SPARK product trees one
    level per launch (SPG_TREE_TOP=0) or every level in the per-circuit workgroup launch; the device Bullet proofs' delta
    on the bucket MSM (SPG_DELTA_COMB=0) instead of the comb parts"""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    case = "mem_both_b3_x64_q2"
    code = (
        "import sys, hashlib; sys.path[:0] = [%r, %r]\n"
        "import spg, workload\n"
        "from r1cs_cases import SNARK_CASES\n"
        "from test_gpu_snark import gpu_snark, GENS_LABEL, GENS_NV\n"
        "ctx = spg.Context(0)\n"
        "g = spg.R1CSGens(ctx, GENS_LABEL, GENS_NV)\n"
        "(p,) = gpu_snark(ctx, g, workload.SnarkWorkload(**SNARK_CASES[%r]), workload.tape_seed())\n"
        "print(hashlib.sha256(p).hexdigest())\n"
    ) % (os.path.join(root, "spartan-parallel_amd"), os.path.join(root, "tests"), case)
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **ROUND_FORMS[form]),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    golden = json.load(open(os.path.join(G, "snark_proofs.json")))[case]
    assert out.stdout.split()[-1] == golden["proof_sha256"]


@pytest.mark.parametrize("host_max,comb", [("0", "1"), ("0", "0"), ("4096", "1")])
def test_bullet_paths(host_max, comb):
    """every DotProductProofLog through the device Bullet rounds (SPG_BULLET_HOST_MAX=0) -- in the comb form
    (k_bullet_comb, the default) or the bucket form (SPG_BULLET_COMB=0, k_bullet_round_q) -- or every one on the
    host pool (4096): the same bytes as the golden proof (a fresh process reads the switches)"""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    case = "mem_both_b3_x64_q2"
    code = (
        "import sys, hashlib; sys.path[:0] = [%r, %r]\n"
        "import spg, workload\n"
        "from r1cs_cases import SNARK_CASES\n"
        "from test_gpu_snark import gpu_snark, GENS_LABEL, GENS_NV\n"
        "ctx = spg.Context(0)\n"
        "g = spg.R1CSGens(ctx, GENS_LABEL, GENS_NV)\n"
        "(p,) = gpu_snark(ctx, g, workload.SnarkWorkload(**SNARK_CASES[%r]), workload.tape_seed())\n"
        "print(hashlib.sha256(p).hexdigest())\n"
    ) % (os.path.join(root, "spartan-parallel_amd"), os.path.join(root, "tests"), case)
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SPG_BULLET_HOST_MAX=host_max,
                                                               SPG_BULLET_COMB=comb),
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    golden = json.load(open(os.path.join(G, "snark_proofs.json")))[case]
    assert out.stdout.split()[-1] == golden["proof_sha256"]
