"""The kernels on a prove's per-round path keep no private (scratch) segment.

Round 4 found the phase-1 / phase-2 quad evaluation kernels with 228 / 292 bytes of scratch per lane (a select of
whole Fq structs, lambdas capturing by-value kernel arguments); removing it cut their device time by a fifth
(DESIGN §4, round 4). This reads the AMDGPU metadata of the built libspg.so's gfx950 code objects
(`.private_segment_fixed_size` per kernel) and fails if a per-round kernel grew one again. CPU only: it reads the
build, it runs nothing on a GPU.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "spartan-parallel_amd", "lib", "libspg.so")
LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
READELF = os.path.join(LLVM, "llvm-readelf")

# kernels every sumcheck / layer / Bullet round launches, and the commit kernels of every prove
HOT = ("k_phase1_eval", "k_phase2_eval", "k_pqx_fold", "k_cubic_eval", "k_eq_table", "k_fold_top",
       "k_layer_round", "k_layer_pair", "k_layer_triple", "k_layer_close", "k_layer_persist", "k_bullet_comb", "k_bullet_round_q", "k_comb_msm_parts",
       "k_smsm_bucket_q", "k_smsm_final", "k_gather_res", "k_spmv", "k_z_fill", "k_abc", "k_bound_part_multi",
       "k_sum_cols_multi", "k_seg_dot", "k_bound_rows", "k_tree_level", "k_tree_top", "k_hash_ops", "k_hash_mem")


def private_segments(tmp_path, field="private_segment_fixed_size"):
    if not (os.path.exists(LIB) and os.path.exists(BUNDLER) and os.path.exists(READELF) and shutil.which("objcopy")):
        pytest.skip("needs the built libspg.so and the ROCm llvm tools")
    fat = tmp_path / "fat.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fat)], check=True)
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = [m.start() for m in re.finditer(re.escape(magic), data)]
    assert offs, "no offload bundle in libspg.so"
    sizes = {}
    for i, o in enumerate(offs):
        part = tmp_path / f"b{i}.bin"
        part.write_bytes(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        co = tmp_path / f"b{i}.co"
        r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode:
            continue
        notes = subprocess.run([READELF, "--notes", str(co)], capture_output=True, text=True, check=True).stdout
        for blk in notes.split("  - .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk)
            ps = re.search(r"\." + field + r":\s+(\d+)", blk)
            if name and ps:
                sizes[name.group(1)] = int(ps.group(1))
    return sizes


def test_round_kernels_have_no_scratch(tmp_path):
    sizes = private_segments(tmp_path)
    hot = {k: v for k, v in sizes.items() if any(h in k for h in HOT)}
    assert len(hot) >= 20, sorted(sizes)[:20]
    assert any("k_phase1_eval_q" in k for k in hot) and any("k_bullet_comb" in k for k in hot)
    bad = {k: v for k, v in hot.items() if v}
    assert not bad, bad


def test_evaluation_kernels_lds(tmp_path):
    """the thread-per-point R1CSProof evaluations reduce through wave shuffles and a few hundred bytes of LDS (a
    24.6 KB LDS tree capped them at 6 workgroups per CU)"""
    lds = private_segments(tmp_path, "group_segment_fixed_size")
    ev = {k: v for k, v in lds.items() if re.search(r"k_phase[12]_evalILb[01]E", k)}
    assert len(ev) >= 4, sorted(lds)[:20]
    assert max(ev.values()) <= 4096, ev
