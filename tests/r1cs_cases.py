"""Shared R1CSProof parity cases (shape only; the data comes from workload.R1CSWorkload).
(num_cons per instance, num_proofs per instance, witness sections, shared instance)"""
CASES = {
    "p2_x4_q2": ([4, 4], [2, 2], 1, False),
    "p3_ragged_3secs": ([8, 4, 2], [4, 2, 1], 3, False),
    "p2_q_single_5secs": ([16, 16], [8, 1], 5, False),
    "shared_p2": ([64, 64], [16, 16], 1, True),
    "p2_x256_2secs": ([256, 256], [64, 64], 2, False),
    "p1_x32": ([32], [8], 1, False),
    "p4_ragged_8secs": ([32, 16, 8, 4], [8, 4, 2, 1], 8, False),
    "p5_q1": ([8, 8, 8, 8, 8], [1, 1, 1, 1, 1], 2, False),
}
# larger shapes checked on the GPU only (oracle still finishes in seconds)
GPU_CASES = {
    "p2_x1024_q64": ([1024, 1024], [64, 64], 1, False),
    "p8_x256_q32_shared": ([256] * 8, [32] * 8, 1, True),
    # more instances than fit in one launch's kernel arguments (kMaxP = 32): descriptors in device memory
    "p40_ragged_2secs": ([16, 8, 32, 8] * 10, [4, 2, 1, 8] * 10, 2, False),
    "p36_shared": ([16] * 36, [2] * 36, 1, True),
}
# SPARK (SparseMatPolyEvalProof) cases: the batch is [A_0, B_0, C_0, A_1, ...] of the workload's instance
SPARK_CASES = {
    "p1_x16": ([16], [4], 1, False),
    "p2_x64_2secs": ([64, 64], [8, 8], 2, False),
    "shared_x32": ([32, 32, 32], [4, 4, 4], 1, True),
    "p2_x256": ([256, 256], [4, 4], 1, False),
}
GPU_SPARK_CASES = {
    "p2_x4096": ([4096, 4096], [2, 2], 1, False),
}

# SNARK::prove cases (workload.SnarkWorkload kwargs): block types, 2^log_cons rows, 2^log_proofs executions each
SNARK_CASES = {
    "b2_x32_q2": dict(num_blocks=2, log_cons=5, log_proofs=1, num_vars=32),
    "b3_x32_q4": dict(num_blocks=3, log_cons=5, log_proofs=2, num_vars=32),
    "b2_x64_q8": dict(num_blocks=2, log_cons=6, log_proofs=3, num_vars=64),
    # memory programs: physical reads of the input stack, virtual store/load pairs (needs niu >= 5), both
    "mem_phy_b2_x64_q4": dict(num_blocks=2, log_cons=6, log_proofs=2, num_vars=64, phy_ops=2, init_phy=5),
    "mem_vir_b2_x64_q4": dict(num_blocks=2, log_cons=6, log_proofs=2, num_vars=64, vir_ops=2, init_vir=3, niu=5),
    "mem_both_b3_x64_q2": dict(num_blocks=3, log_cons=6, log_proofs=1, num_vars=64, phy_ops=1, vir_ops=2, init_phy=3,
                               init_vir=5, niu=5),
    # uneven traces: block_num_proofs not sorted ([2, 4, 0]), a block that never runs, num_proofs = 1, per-block
    # witness widths (num_vars_per_block) below num_vars
    "uneven_b3_x32": dict(num_blocks=3, log_cons=5, log_proofs=1, num_vars=32, schedule=[0, 1, 1, 1, 0, 1]),
    "widths_b3_x64": dict(num_blocks=3, log_cons=5, log_proofs=1, num_vars=64, vars_width=[64, 32, 32],
                          schedule=[0, 1, 1, 2, 1]),
    "mem_uneven_b3_x64": dict(num_blocks=3, log_cons=6, log_proofs=1, num_vars=64, phy_ops=1, vir_ops=2, init_phy=3,
                              init_vir=5, niu=5, schedule=[2, 0, 2, 2, 0, 2]),
}
GPU_SNARK_CASES = {
    "b34_x32_q2": dict(num_blocks=34, log_cons=5, log_proofs=1, num_vars=32),  # > 32 block types (kMaxP)
    "b2_x1024_q8": dict(num_blocks=2, log_cons=10, log_proofs=3, num_vars=1024),
    # SURVEY 8d config 1 exactly: 2 block types x 2 executions x 2^10 constraints (2^12), num_vars 2^10
    "b2_x1024_q2": dict(num_blocks=2, log_cons=10, log_proofs=1, num_vars=1024),
    "b2_x256_q64": dict(num_blocks=2, log_cons=8, log_proofs=6, num_vars=256),
    "mem_both_b2_x256_q32": dict(num_blocks=2, log_cons=8, log_proofs=5, num_vars=256, phy_ops=3, vir_ops=2,
                                 init_phy=20, init_vir=7, niu=5),
}
ALL_R1CS = dict(CASES, **GPU_CASES)
