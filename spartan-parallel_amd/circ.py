"""CirC front-end files -> SNARK::prove on the GPU (the host side of examples/interface.rs).

CirC writes two bincode files per program: `{name}_bin.ctk` (CompileTimeKnowledge: the block circuits and the
program shape, examples/interface.rs:45-71) and `{name}_bin.rtk` (RunTimeKnowledge: the execution trace and memory
lists, :195-216). bincode 1.x with serde derive: fields in declaration order, usize as u64 LE, Vec<T> as a u64 length
then the elements, [u8; 32] as 32 raw bytes, bool as one byte, tuples field by field; an Assignment
(src/lib.rs:87-92) is its Vec<Scalar>, and a Scalar serialises as its four u64 Montgomery limbs
(src/scalar/ristretto255.rs:198) — the same layout libspg takes, so witness data passes through untouched.

`CircProgram(ctk, rtk)` restates interface.rs:458-563: the block instances from the CTK's constraint terms
(Instance::gen_block_inst), the pairwise-check and permutation-root instances, the SNARKGens sizes, and the
SNARK::prove inputs; it exposes the attributes `workload.SnarkViews` reads, so the same views feed libspg (and, in
the tests, the CPU oracle). `prove()` runs the device prover; `python circ.py NAME --dir zok_tests` mirrors the
example binary (files at `{dir}/constraints/{NAME}_bin.ctk` and `{dir}/inputs/{NAME}_bin.rtk`).
"""
import argparse
import dataclasses
import os
import struct
import sys
import time
from typing import List, Tuple

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import workload  # noqa: E402

Q = workload.Q
TOTAL_NUM_VARS_BOUND = 10000000  # examples/interface.rs:15

Term = Tuple[int, bytes]  # (variable index, 32-byte little-endian canonical scalar)


class _Reader:
    def __init__(self, b):
        self.b = memoryview(b)
        self.o = 0

    def u64(self):
        if self.o + 8 > len(self.b):
            raise ValueError("bincode: truncated input")
        v = struct.unpack_from("<Q", self.b, self.o)[0]
        self.o += 8
        return v

    def boolean(self):
        if self.o >= len(self.b):
            raise ValueError("bincode: truncated input")
        v = self.b[self.o]
        self.o += 1
        if v > 1:
            raise ValueError(f"bincode: invalid bool byte {v} at offset {self.o - 1}")
        return bool(v)

    def raw(self, n):
        if self.o + n > len(self.b):
            raise ValueError("bincode: truncated input")
        v = bytes(self.b[self.o:self.o + n])
        self.o += n
        return v

    def vec(self, item):
        return [item() for _ in range(self.u64())]

    def usizes(self):
        n = self.u64()
        if self.o + 8 * n > len(self.b):
            raise ValueError("bincode: truncated input")
        v = np.frombuffer(self.b, dtype="<u8", count=n, offset=self.o).astype(np.int64).tolist()
        self.o += 8 * n
        return v

    def assignment(self):
        """Assignment { assignment: Vec<Scalar> } -> (n, 4) uint64 Montgomery limbs"""
        n = self.u64()
        if self.o + 32 * n > len(self.b):
            raise ValueError("bincode: truncated input")
        a = np.frombuffer(self.b, dtype="<u8", count=4 * n, offset=self.o).astype(np.uint64).reshape(n, 4)
        self.o += 32 * n
        return a

    def end(self):
        if self.o != len(self.b):
            raise ValueError(f"bincode: {len(self.b) - self.o} trailing bytes")


class _Writer:
    def __init__(self):
        self.parts = []

    def u64(self, v):
        self.parts.append(struct.pack("<Q", int(v)))

    def boolean(self, v):
        self.parts.append(b"\x01" if v else b"\x00")

    def raw(self, b):
        self.parts.append(bytes(b))

    def usizes(self, v):
        self.u64(len(v))
        self.parts.append(np.asarray(v, dtype="<u8").tobytes())

    def assignment(self, a):
        a = np.ascontiguousarray(a, dtype="<u8").reshape(-1, 4)
        self.u64(a.shape[0])
        self.parts.append(a.tobytes())

    def bytes(self):
        return b"".join(self.parts)


def _terms_read(r):
    return r.vec(lambda: (r.u64(), r.raw(32)))


def _terms_write(w, terms):
    w.u64(len(terms))
    for col, val in terms:
        w.u64(col)
        w.raw(val)


@dataclasses.dataclass
class CompileTimeKnowledge:
    """examples/interface.rs:45-71 (field order = bincode order)"""
    block_num_instances: int
    num_vars: int
    num_inputs_unpadded: int
    num_vars_per_block: List[int]
    block_num_phy_ops: List[int]
    block_num_vir_ops: List[int]
    max_ts_width: int
    args: List[List[Tuple[List[Term], List[Term], List[Term]]]]
    input_liveness: List[bool]
    func_input_width: int
    input_offset: int
    input_block_num: int
    output_offset: int
    output_block_num: int

    @classmethod
    def from_bytes(cls, b):
        r = _Reader(b)
        v = dict(block_num_instances=r.u64(), num_vars=r.u64(), num_inputs_unpadded=r.u64(),
                 num_vars_per_block=r.usizes(), block_num_phy_ops=r.usizes(), block_num_vir_ops=r.usizes(),
                 max_ts_width=r.u64())
        v["args"] = r.vec(lambda: r.vec(lambda: (_terms_read(r), _terms_read(r), _terms_read(r))))
        v["input_liveness"] = r.vec(r.boolean)
        for f in ("func_input_width", "input_offset", "input_block_num", "output_offset", "output_block_num"):
            v[f] = r.u64()
        r.end()
        return cls(**v)

    def to_bytes(self):
        w = _Writer()
        for f in ("block_num_instances", "num_vars", "num_inputs_unpadded"):
            w.u64(getattr(self, f))
        for f in ("num_vars_per_block", "block_num_phy_ops", "block_num_vir_ops"):
            w.usizes(getattr(self, f))
        w.u64(self.max_ts_width)
        w.u64(len(self.args))
        for block in self.args:
            w.u64(len(block))
            for a, b, c in block:
                _terms_write(w, a)
                _terms_write(w, b)
                _terms_write(w, c)
        w.u64(len(self.input_liveness))
        for x in self.input_liveness:
            w.boolean(x)
        for f in ("func_input_width", "input_offset", "input_block_num", "output_offset", "output_block_num"):
            w.u64(getattr(self, f))
        return w.bytes()


@dataclasses.dataclass
class RunTimeKnowledge:
    """examples/interface.rs:195-216 (field order = bincode order); assignments as (n, 4) uint64 Montgomery limbs,
    byte fields as 32-byte little-endian canonical scalars"""
    block_max_num_proofs: int
    block_num_proofs: List[int]
    consis_num_proofs: int
    total_num_init_phy_mem_accesses: int
    total_num_init_vir_mem_accesses: int
    total_num_phy_mem_accesses: int
    total_num_vir_mem_accesses: int
    block_vars_matrix: List[List[np.ndarray]]
    exec_inputs: List[np.ndarray]
    init_phy_mems_list: List[np.ndarray]
    init_vir_mems_list: List[np.ndarray]
    addr_phy_mems_list: List[np.ndarray]
    addr_vir_mems_list: List[np.ndarray]
    addr_ts_bits_list: List[np.ndarray]
    input: List[bytes]
    input_stack: List[bytes]
    input_mem: List[bytes]
    output: bytes
    output_exec_num: int

    _LISTS = ("exec_inputs", "init_phy_mems_list", "init_vir_mems_list", "addr_phy_mems_list", "addr_vir_mems_list",
              "addr_ts_bits_list")
    _COUNTS = ("consis_num_proofs", "total_num_init_phy_mem_accesses", "total_num_init_vir_mem_accesses",
               "total_num_phy_mem_accesses", "total_num_vir_mem_accesses")

    @classmethod
    def from_bytes(cls, b):
        r = _Reader(b)
        v = dict(block_max_num_proofs=r.u64(), block_num_proofs=r.usizes())
        for f in cls._COUNTS:
            v[f] = r.u64()
        v["block_vars_matrix"] = r.vec(lambda: r.vec(r.assignment))
        for f in cls._LISTS:
            v[f] = r.vec(r.assignment)
        for f in ("input", "input_stack", "input_mem"):
            v[f] = r.vec(lambda: r.raw(32))
        v["output"] = r.raw(32)
        v["output_exec_num"] = r.u64()
        r.end()
        return cls(**v)

    def to_bytes(self):
        w = _Writer()
        w.u64(self.block_max_num_proofs)
        w.usizes(self.block_num_proofs)
        for f in self._COUNTS:
            w.u64(getattr(self, f))
        w.u64(len(self.block_vars_matrix))
        for rows in self.block_vars_matrix:
            w.u64(len(rows))
            for a in rows:
                w.assignment(a)
        for f in self._LISTS:
            rows = getattr(self, f)
            w.u64(len(rows))
            for a in rows:
                w.assignment(a)
        for f in ("input", "input_stack", "input_mem"):
            rows = getattr(self, f)
            w.u64(len(rows))
            for x in rows:
                w.raw(x)
        w.raw(self.output)
        w.u64(self.output_exec_num)
        return w.bytes()


def scalar_from_bytes(b):
    """Scalar::from_bytes (canonical little-endian; a value >= q is R1CSError::InvalidScalar, src/lib.rs:96-108)"""
    v = int.from_bytes(b, "little")
    if v >= Q:
        raise ValueError("InvalidScalar: a 32-byte scalar is not canonical")
    return v


def scalar_to_bytes(v):
    return (int(v) % Q).to_bytes(32, "little")


def _mont_rows(rows, width, what):
    """a list of Assignments (each (width, 4)) -> (n, width, 4) uint64"""
    if not rows:
        return np.zeros((0, width, 4), dtype=np.uint64)
    for a in rows:
        if a.shape[0] != width:
            raise ValueError(f"{what}: assignment of {a.shape[0]} entries, expected {width}")
    return np.ascontiguousarray(np.stack(rows), dtype=np.uint64)


class CircProgram:
    """SNARK::prove inputs of one CirC program (examples/interface.rs:458-563); attribute names follow
    workload.SnarkWorkload, which `workload.SnarkViews` turns into the libspg C structs."""

    def __init__(self, ctk: CompileTimeKnowledge, rtk: RunTimeKnowledge):
        B = ctk.block_num_instances
        # interface.rs:463-479
        if ctk.num_vars & (ctk.num_vars - 1):
            raise ValueError("num_vars must be a power of two")
        if not (len(ctk.args) == B and len(ctk.block_num_phy_ops) == B and len(ctk.block_num_vir_ops) == B
                and len(ctk.num_vars_per_block) == B and len(rtk.block_num_proofs) == B):
            raise ValueError("per-block lists must have block_num_instances entries")
        if ctk.output_block_num < B:
            raise ValueError("output_block_num must be at least block_num_instances")
        self.num_blocks = B
        self.num_vars = ctk.num_vars
        self.num_inputs_unpadded = niu = ctk.num_inputs_unpadded
        self.num_ios = 1 << (2 * niu - 1).bit_length()
        self.block_num_phy_ops = list(ctk.block_num_phy_ops)
        self.block_num_vir_ops = list(ctk.block_num_vir_ops)
        self.max_ts_width = ctk.max_ts_width
        self.mem_addr_ts_bits_size = 1 << (2 + ctk.max_ts_width - 1).bit_length()
        self._num_vars_per_block = list(ctk.num_vars_per_block)
        # Instance::gen_block_inst / gen_pairwise_check_inst / gen_perm_root_inst (interface.rs:482-518)
        args = [[tuple([(col, scalar_from_bytes(v)) for col, v in terms] for terms in row) for row in block]
                for block in ctk.args]
        self.block_num_vars, self.block_max_num_cons, self.block_nnz, self.block_inst = workload.gen_block_inst(
            ctk.num_vars, args, niu, self.block_num_phy_ops, self.block_num_vir_ops)
        (self.pairwise_num_vars, self.pairwise_max_num_cons, self.pairwise_nnz,
         self.pairwise_inst) = workload.gen_pairwise_check_inst(ctk.max_ts_width, self.mem_addr_ts_bits_size)
        self.perm_root_num_cons, self.perm_root_nnz, self.perm_root_inst = workload.gen_perm_root_inst(
            niu, self.num_ios)
        # run-time inputs (interface.rs:535-563 -> SNARK::prove, src/lib.rs:971-1026)
        self.block_num_proofs = list(rtk.block_num_proofs)
        self.block_max_num_proofs = rtk.block_max_num_proofs
        if max(self.block_num_proofs) > self.block_max_num_proofs:
            raise ValueError("block_num_proofs exceeds block_max_num_proofs")
        order = sorted(range(B), key=lambda b: -self.block_num_proofs[b])
        executed = [b for b in order if self.block_num_proofs[b] > 0]
        if len(rtk.block_vars_matrix) != len(executed):
            raise ValueError("block_vars_matrix must hold one list per executed block (in the prover's sort order)")
        self._block_vars_sorted = []
        for i, b in enumerate(executed):
            rows = rtk.block_vars_matrix[i]
            if len(rows) != self.block_num_proofs[b]:
                raise ValueError(f"block_vars_matrix[{i}]: {len(rows)} executions, block {b} has "
                                 f"{self.block_num_proofs[b]}")
            self._block_vars_sorted.append(_mont_rows(rows, self._num_vars_per_block[b], f"block_vars_matrix[{i}]"))
        self._block_vars_sorted += [np.zeros((0, self._num_vars_per_block[b], 4), dtype=np.uint64)
                                    for b in order[len(executed):]]
        self.consis_num_proofs = rtk.consis_num_proofs
        if len(rtk.exec_inputs) != rtk.consis_num_proofs:
            raise ValueError("exec_inputs must hold consis_num_proofs assignments")
        self.exec_inputs = _mont_rows(rtk.exec_inputs, self.num_ios, "exec_inputs")
        lists = (("init_phy_mems", rtk.init_phy_mems_list, rtk.total_num_init_phy_mem_accesses, 4),
                 ("init_vir_mems", rtk.init_vir_mems_list, rtk.total_num_init_vir_mem_accesses, 4),
                 ("addr_phy_mems", rtk.addr_phy_mems_list, rtk.total_num_phy_mem_accesses, 4),
                 ("addr_vir_mems", rtk.addr_vir_mems_list, rtk.total_num_vir_mem_accesses, 8),
                 ("addr_ts_bits", rtk.addr_ts_bits_list, rtk.total_num_vir_mem_accesses, self.mem_addr_ts_bits_size))
        for name, rows, total, width in lists:
            if len(rows) != total:
                raise ValueError(f"{name}: {len(rows)} entries, expected {total}")
            setattr(self, name, _mont_rows(rows, width, name))
        self.input_block_num = ctk.input_block_num
        self.output_block_num = ctk.output_block_num
        self.input_liveness = list(ctk.input_liveness)
        self.func_input_width = ctk.func_input_width
        self.input_offset = ctk.input_offset
        self.output_offset = ctk.output_offset
        self.input = workload.to_mont_limbs([scalar_from_bytes(x) for x in rtk.input])
        self.output_mont = workload.to_mont_limbs([scalar_from_bytes(rtk.output)])[0]
        self.output_exec_num = rtk.output_exec_num

    @property
    def num_vars_per_block(self):
        return self._num_vars_per_block

    @property
    def block_vars_sorted(self):
        return self._block_vars_sorted

    @property
    def total_constraints(self):
        npow = lambda v: 1 << max(0, (v - 1).bit_length())
        return sum(npow(q) * c for q, c in zip(self.block_num_proofs, self.block_inst[2]) if q)

    @classmethod
    def load(cls, ctk_path, rtk_path):
        with open(ctk_path, "rb") as f:
            ctk = CompileTimeKnowledge.from_bytes(f.read())
        with open(rtk_path, "rb") as f:
            rtk = RunTimeKnowledge.from_bytes(f.read())
        return cls(ctk, rtk)


def export_workload(wl):
    """a workload.SnarkWorkload as the (CompileTimeKnowledge, RunTimeKnowledge) CirC would write for it"""
    B = wl.num_blocks
    args = [[tuple([(col, scalar_to_bytes(v)) for col, v in terms] for terms in row) for row in block]
            for block in wl.args]
    ctk = CompileTimeKnowledge(
        block_num_instances=B, num_vars=wl.num_vars, num_inputs_unpadded=wl.num_inputs_unpadded,
        num_vars_per_block=list(wl.num_vars_per_block), block_num_phy_ops=list(wl.block_num_phy_ops),
        block_num_vir_ops=list(wl.block_num_vir_ops), max_ts_width=wl.max_ts_width, args=args,
        input_liveness=list(wl.input_liveness), func_input_width=wl.func_input_width, input_offset=wl.input_offset,
        input_block_num=wl.input_block_num, output_offset=wl.output_offset, output_block_num=wl.output_block_num)

    def mont(rows):
        if isinstance(rows, np.ndarray) and rows.dtype == np.uint64:
            return [np.asarray(r) for r in rows]
        return [workload.to_mont_limbs(r) for r in rows]

    def canon(m):  # Montgomery limbs -> 32-byte canonical
        v = sum(int(m[i]) << (64 * i) for i in range(4))
        return scalar_to_bytes(v * pow(workload.R, -1, Q))

    rtk = RunTimeKnowledge(
        block_max_num_proofs=wl.block_max_num_proofs, block_num_proofs=list(wl.block_num_proofs),
        consis_num_proofs=wl.consis_num_proofs,
        total_num_init_phy_mem_accesses=len(wl.init_phy_mems), total_num_init_vir_mem_accesses=len(wl.init_vir_mems),
        total_num_phy_mem_accesses=len(wl.addr_phy_mems), total_num_vir_mem_accesses=len(wl.addr_vir_mems),
        block_vars_matrix=[list(v) for v in wl.block_vars_sorted if len(v)],
        exec_inputs=list(wl.exec_inputs), init_phy_mems_list=mont(wl.init_phy_mems),
        init_vir_mems_list=mont(wl.init_vir_mems), addr_phy_mems_list=mont(wl.addr_phy_mems),
        addr_vir_mems_list=mont(wl.addr_vir_mems), addr_ts_bits_list=mont(wl.addr_ts_bits),
        input=[canon(m) for m in wl.input], input_stack=[scalar_to_bytes(v) for v in wl.input_stack],
        input_mem=[scalar_to_bytes(v) for v in wl.input_mem], output=canon(wl.output_mont),
        output_exec_num=wl.output_exec_num)
    return ctk, rtk


def prove(ctx, prog, tape_seed=None, label=b"snark_example", vars_gens=None):
    """SNARK::prove of a CircProgram on the device (interface.rs:520-597): returns bincode(SNARK)"""
    import spg

    views = workload.SnarkViews(prog)
    gens = vars_gens or spg.R1CSGens(ctx, b"gens_r1cs_sat", TOTAL_NUM_VARS_BOUND)
    block = spg.SnarkComp(ctx, views.block, multi=True)
    pairwise = spg.SnarkComp(ctx, views.pairwise)
    perm_root = spg.SnarkComp(ctx, views.perm_root)
    wit = spg.SnarkWitness(ctx, views.inputs)
    seed = workload.tape_seed() if tape_seed is None else tape_seed
    return spg.snark_prove(ctx, block, pairwise, perm_root, wit, gens, spg.Transcript(label),
                           spg.RandomTape(b"proof", seed))


def main(argv=None):
    ap = argparse.ArgumentParser(description="SNARK::prove of a CirC program (examples/interface.rs)")
    ap.add_argument("benchmark_name")
    ap.add_argument("--dir", default="../zok_tests", help="directory holding constraints/ and inputs/")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", default=None, help="write bincode(SNARK) here")
    a = ap.parse_args(argv)
    import spg

    t0 = time.perf_counter()
    prog = CircProgram.load(os.path.join(a.dir, "constraints", f"{a.benchmark_name}_bin.ctk"),
                            os.path.join(a.dir, "inputs", f"{a.benchmark_name}_bin.rtk"))
    ctx = spg.Context(a.device)
    gens = spg.R1CSGens(ctx, b"gens_r1cs_sat", TOTAL_NUM_VARS_BOUND)
    print(f"Preprocess time: {1e3 * (time.perf_counter() - t0):.0f}ms")
    t1 = time.perf_counter()
    proof = prove(ctx, prog, vars_gens=gens)
    dt = time.perf_counter() - t1
    print(f"Proof time: {1e3 * dt:.1f}ms ({prog.total_constraints} constraints, {len(proof)} proof bytes)")
    if a.out:
        with open(a.out, "wb") as f:
            f.write(proof)


if __name__ == "__main__":
    main()
