"""ctypes wrapper of the C oracle (keto_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / CPU baseline.  The product (keto_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libketo_oracle.so")

POLICY_CANONICAL = 0
POLICY_DFS = 1
N, M, ERR = 0, 1, 2
SUBJECT_ID = 0xFFFFFFFF
SET_BIT = 0x80000000


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, u32, u64, i32, i64 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32, C.c_int64
        L.ko_index_new.restype = vp
        L.ko_index_new.argtypes = [u32, u32]
        L.ko_index_free.argtypes = [vp]
        L.ko_index_add_tuples.argtypes = [vp, vp, u64]
        L.ko_index_finalize.argtypes = [vp]
        L.ko_index_from_csr.restype = vp
        L.ko_index_from_csr.argtypes = [u32, u32, vp, vp, vp, vp, vp, C.c_int, C.c_int]
        L.ko_index_n_nodes.restype = u32
        L.ko_index_n_nodes.argtypes = [vp]
        L.ko_index_n_rows.restype = u64
        L.ko_index_n_rows.argtypes = [vp]
        L.ko_set_program.argtypes = [vp, u32, vp, u32, vp, vp, vp, u32, vp, u32, vp]
        L.ko_check.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.POINTER(i32)]
        L.ko_check_batch.argtypes = [vp, vp, vp, u64, C.c_int, C.c_int, C.c_int, vp, vp, vp]
        L.ko_check_nodes_batch.argtypes = [vp, vp, vp, vp, u64, C.c_int, C.c_int, C.c_int, vp, vp]
        L.ko_expand.restype = i64
        L.ko_expand.argtypes = [vp, u32, u32, u32, C.c_int, C.c_int, vp, i64]
        L.ko_expand_node.restype = i64
        L.ko_expand_node.argtypes = [vp, u32, C.c_int, C.c_int, vp, i64]
        L.ko_expand_nodes_batch.argtypes = [vp, vp, vp, u64, C.c_int, C.c_int, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Row index + namespace program, queried with interned ids."""

    def __init__(self, tuples: Optional[np.ndarray], wildcard_rel: int, program=None, page_size: int = 100,
                 _handle=None):
        L = lib()
        if _handle is not None:
            self.h = _handle
        else:
            self.h = L.ko_index_new(wildcard_rel, page_size)
            t = np.ascontiguousarray(tuples, dtype=np.uint32).reshape(-1, 6)
            L.ko_index_add_tuples(self.h, _p(t), t.shape[0])
            L.ko_index_finalize(self.h)
        self._keep = []
        if program is not None:
            self.set_program(program)

    @classmethod
    def from_csr(cls, wildcard_rel, nd_ns, nd_obj, nd_rel, row_off, row_subj, with_node_map=False,
                 nthreads=1) -> "Oracle":
        L = lib()
        arrs = [np.ascontiguousarray(a, dtype=np.uint32) for a in (nd_ns, nd_obj, nd_rel)]
        off = np.ascontiguousarray(row_off, dtype=np.uint64)
        sub = np.ascontiguousarray(row_subj, dtype=np.uint32)
        h = L.ko_index_from_csr(wildcard_rel, len(arrs[0]), _p(arrs[0]), _p(arrs[1]), _p(arrs[2]), _p(off), _p(sub),
                                int(with_node_map), int(nthreads))
        return cls(None, wildcard_rel, _handle=h)

    def set_program(self, prog) -> None:
        arrs = [np.ascontiguousarray(prog.ns_has_rel, np.uint8), np.ascontiguousarray(prog.rel_ns, np.uint32),
                np.ascontiguousarray(prog.rel_rel, np.uint32), np.ascontiguousarray(prog.rel_root, np.int32),
                np.ascontiguousarray(prog.rw, np.int32).reshape(-1, 5), np.ascontiguousarray(prog.child, np.int32)]
        self._keep = arrs
        lib().ko_set_program(self.h, len(arrs[0]), _p(arrs[0]), len(arrs[1]), _p(arrs[1]), _p(arrs[2]), _p(arrs[3]),
                             arrs[4].shape[0], _p(arrs[4]), len(arrs[5]), _p(arrs[5]))

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().ko_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_nodes(self) -> int:
        return lib().ko_index_n_nodes(self.h)

    def check(self, q6: Sequence[int], max_depth: int, global_max: int, policy: int = POLICY_CANONICAL) -> Tuple[int, int]:
        """Returns (result, err_code): result 0 = not allowed, 1 = allowed, 2 = error."""
        q = np.asarray(q6, dtype=np.uint32).reshape(6)
        err = C.c_int32(0)
        r = lib().ko_check(self.h, _p(q), int(max_depth), int(global_max), int(policy), C.byref(err))
        return int(r), int(err.value)

    def check_batch(self, q: np.ndarray, depths: np.ndarray, global_max: int, policy: int = POLICY_CANONICAL,
                    nthreads: int = 1):
        q = np.ascontiguousarray(q, dtype=np.uint32).reshape(-1, 6)
        d = np.ascontiguousarray(depths, dtype=np.int32)
        out = np.zeros(q.shape[0], np.uint8)
        err = np.zeros(q.shape[0], np.int32)
        st = np.zeros(3, np.uint64)
        lib().ko_check_batch(self.h, _p(q), _p(d), q.shape[0], int(global_max), int(policy), int(nthreads),
                             _p(out), _p(err), _p(st))
        return out, err, st

    def check_nodes_batch(self, node: np.ndarray, subj: np.ndarray, depths: np.ndarray, global_max: int,
                          policy: int = POLICY_DFS, nthreads: int = 1):
        node = np.ascontiguousarray(node, np.uint32)
        subj = np.ascontiguousarray(subj, np.uint32)
        d = np.ascontiguousarray(depths, np.int32)
        out = np.zeros(node.shape[0], np.uint8)
        st = np.zeros(3, np.uint64)
        lib().ko_check_nodes_batch(self.h, _p(node), _p(subj), _p(d), node.shape[0], int(global_max), int(policy),
                                   int(nthreads), _p(out), _p(st))
        return out, st

    def expand(self, sns: int, sobj: int, srel: int, max_depth: int, global_max: int) -> Optional[np.ndarray]:
        """Pre-order records (n, 6) = (type, is_set, ns, obj, rel, n_children), or None for nil."""
        cap = 1024
        while True:
            buf = np.zeros((cap, 6), np.int32)
            n = lib().ko_expand(self.h, sns, sobj, srel, int(max_depth), int(global_max), _p(buf), cap)
            if n >= 0:
                return buf[:n] if n > 0 else None
            cap = -n + 16

    def expand_node(self, node: int, max_depth: int, global_max: int) -> Optional[np.ndarray]:
        """expand of the subject set whose node id is `node` (no node map needed)."""
        if not 0 <= int(node) < self.n_nodes:
            raise ValueError(f"node {node} out of range")
        cap = 1024
        while True:
            buf = np.zeros((cap, 6), np.int32)
            n = lib().ko_expand_node(self.h, int(node), int(max_depth), int(global_max), _p(buf), cap)
            if n >= 0:
                return buf[:n] if n > 0 else None
            cap = -n + 16

    def expand_nodes_batch(self, nodes: np.ndarray, depths: np.ndarray, global_max: int, nthreads: int = 1) -> np.ndarray:
        """expand_node over many roots on `nthreads` threads (ko_expand_nodes_batch); returns each root's
        record count (0 = nil).  The trees themselves are built and dropped (the C5 CPU baseline)."""
        nodes = np.ascontiguousarray(nodes, np.uint32)
        d = np.ascontiguousarray(depths, np.int32)
        if nodes.size and int(nodes.max()) >= self.n_nodes:
            raise ValueError("node out of range")
        counts = np.zeros(nodes.shape[0], np.int64)
        if lib().ko_expand_nodes_batch(self.h, _p(nodes), _p(d), nodes.shape[0], int(global_max), int(nthreads),
                                       _p(counts)) != 0:
            raise MemoryError("ko_expand_nodes_batch")
        return counts


def records_to_tree(rec: Optional[np.ndarray], interner):
    """Convert pre-order records into a keto_amd.ketoapi.Tree (strings)."""
    from keto_amd.ketoapi import Tree, TREE_UNION, TREE_LEAF
    if rec is None or len(rec) == 0:
        return None
    pos = [0]

    def rec_tree():
        r = rec[pos[0]]
        pos[0] += 1
        subj = interner.subject_from_ids(bool(r[1]), int(r[2]), int(r[3]), int(r[4]))
        t = Tree(TREE_UNION if r[0] == 1 else TREE_LEAF, subj)
        for _ in range(int(r[5])):
            t.children.append(rec_tree())
        return t

    return rec_tree()
