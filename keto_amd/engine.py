"""Host-side mirror of the reference's check / expand engine surface, running on the MI355X
library through the C ABI.

Reference interfaces mirrored (paths relative to the reference checkout):
  check.NewEngine / Engine.CheckIsMember / CheckRelationTuple   internal/check/engine.go:42-80
  Engine.BatchCheck (new)                         == a loop of CheckIsMember
  expand.Engine.BuildTree                                       internal/expand/engine.go:35-104
  config.Provider.MaxReadDepth (default 5, 1..65535)            internal/driver/config/provider.go:160-162
  checkgroup.Result{Membership, Tree, Err}                      internal/check/checkgroup/definitions.go:46-69
    (the tree of a member result: keto_amd/explain.py)
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .ketoapi import CheckTree, RelationTuple, SubjectSet, Tree, TREE_LEAF, TREE_UNION
from .mapper import Interner, Mapper, SUBJECT_ID
from .namespace import Namespace, Program, compile_program

MEMBERSHIP_UNKNOWN, IS_MEMBER, NOT_MEMBER = 0, 1, 2  # checkgroup.Membership

ERR_TEXT = {
    _lib.KG_ERR_RELATION_NOT_FOUND: "relation not found",       # engine.go:228
    _lib.KG_ERR_NOT_IMPLEMENTED: "not implemented",             # rewrites.go:15-17
    _lib.KG_ERR_REWRITE_CYCLE: "computed subject-set rewrite cycle",
    _lib.KG_ERR_RESOURCE: "engine capacity exceeded",
}


class CheckError(RuntimeError):
    def __init__(self, code: int):
        super().__init__(ERR_TEXT.get(code, f"error {code}"))
        self.code = code


@dataclass
class Result:
    membership: int
    err: Optional[CheckError] = None
    tree: Optional[CheckTree] = None


@dataclass
class Config:
    max_read_depth: int = 5
    namespaces: List[Namespace] = field(default_factory=list)

    def __post_init__(self):
        if not 1 <= self.max_read_depth <= 65535:  # embedx/config.schema.json:308-315
            raise ValueError("max_read_depth must be in [1, 65535]")


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Snapshot:
    """An HBM-resident, immutable snapshot of the relation tuples (rows in shard order)."""

    def __init__(self, tuples: np.ndarray, interner: Interner, program: Optional[Program] = None, device: int = 0,
                 _handle=None, shard: Optional[Tuple[int, int]] = None, devices: Optional[Sequence[int]] = None,
                 keys: Optional[np.ndarray] = None):
        """devices: one replica per entry (entries may repeat); the library splits host-buffer batches
        over them (kg_snapshot_create_on).  Default: one replica on `device`.
        shard = (rank, nranks): keep only the rows of the nodes this rank owns (hash-sharded mode,
        keto_amd.sharded); every rank passes the same full tuple list.
        keys: ascending u64 order key per row (shard ids): kept so `apply` places inserted rows in order
        (kg_snapshot_create_ordered)."""
        L = _lib.load()
        self.interner = interner
        self.device = device
        self.program = program
        self.shard = shard
        self._keep = []
        self._h = C.c_void_p()
        if _handle is not None:
            self._h = _handle
            return
        t = np.ascontiguousarray(tuples, dtype=np.uint32).reshape(-1, 6)
        d = _lib.kg_dict(interner.n_namespaces, interner.n_relations, interner.wildcard_rel)
        prog_c = self._prog(program)
        pc = C.byref(prog_c) if prog_c is not None else None
        self.devices = list(devices) if devices else [device]
        if shard is None and keys is not None:
            dv = np.asarray(self.devices, np.int32)
            k = np.ascontiguousarray(keys, dtype=np.uint64)
            rc = L.kg_snapshot_create_ordered(_ptr(t), _ptr(k), t.shape[0], C.byref(d), pc, _ptr(dv), len(dv),
                                              C.byref(self._h))
        elif shard is None:
            dv = np.asarray(self.devices, np.int32)
            rc = L.kg_snapshot_create_on(_ptr(t), t.shape[0], C.byref(d), pc, _ptr(dv), len(dv), C.byref(self._h))
        else:
            rc = L.kg_snapshot_create_shard(_ptr(t), t.shape[0], C.byref(d), pc, device, shard[0], shard[1],
                                            C.byref(self._h))
        _lib.check(rc, "kg_snapshot_create")

    def _prog(self, program: Optional[Program]):
        self._keep = []
        if program is None or program.empty:
            return None
        arrs = [np.ascontiguousarray(program.ns_has_rel, np.uint8), np.ascontiguousarray(program.rel_ns, np.uint32),
                np.ascontiguousarray(program.rel_rel, np.uint32), np.ascontiguousarray(program.rel_root, np.int32),
                np.ascontiguousarray(program.rw, np.int32).reshape(-1, 5), np.ascontiguousarray(program.child, np.int32)]
        self._keep = arrs
        return _lib.kg_rewrite_prog(len(arrs[0]), _ptr(arrs[0]), len(arrs[1]), _ptr(arrs[1]), _ptr(arrs[2]),
                                    _ptr(arrs[3]), arrs[4].shape[0], _ptr(arrs[4]), len(arrs[5]), _ptr(arrs[5]))

    def apply(self, ins: np.ndarray, dels: np.ndarray, ins_keys: Optional[np.ndarray] = None) -> "Snapshot":
        """kg_snapshot_apply: a new snapshot holding this one's rows minus every row equal to a tuple of
        `dels`, plus `ins` (uint32 (n, 6) tuple ids; ins_keys: their order keys).  This snapshot stays
        valid for readers; the next delta goes to the returned one."""
        L = _lib.load()
        it = self.interner
        a = np.ascontiguousarray(ins, dtype=np.uint32).reshape(-1, 6)
        dl = np.ascontiguousarray(dels, dtype=np.uint32).reshape(-1, 6)
        k = None if ins_keys is None else np.ascontiguousarray(ins_keys, dtype=np.uint64)
        d = _lib.kg_dict(it.n_namespaces, it.n_relations, it.wildcard_rel)
        new = Snapshot(None, it, self.program, self.device, _handle=C.c_void_p())
        prog_c = new._prog(self.program)
        pc = C.byref(prog_c) if prog_c is not None else None
        h = C.c_void_p()
        _lib.check(L.kg_snapshot_apply(self._h, _ptr(a) if len(a) else None, _ptr(k) if k is not None and len(a) else None,
                                       a.shape[0], _ptr(dl) if len(dl) else None, dl.shape[0], C.byref(d), pc,
                                       C.byref(h)), "kg_snapshot_apply")
        new._h = h
        new.devices = getattr(self, "devices", [self.device])
        return new

    @classmethod
    def synthetic(cls, n_tuples: int, seed: int = 20250131, device: int = 0, n_layers: int = 8,
                  max_degree: int = 100000, set_fraction: float = 0.25, doc_set_fraction: float = 0.5,
                  preset: int = 0, shard: Optional[Tuple[int, int]] = None,
                  devices: Optional[Sequence[int]] = None, doc_alpha: float = 0.0,
                  group_alpha: float = 0.0) -> "Snapshot":
        """Device-generated Drive-like graph (keto_amd/csrc/kg_synth.h); preset 0 = C2/C4, 1 = C3.
        shard = (rank, nranks): only this rank's rows (hash-sharded mode)."""
        from . import synth
        L = _lib.load()
        it = synth.interner()
        prog = synth.program(preset, it)
        snap = cls(None, it, device=device, _handle=C.c_void_p())
        p = _lib.kg_synth_params(n_tuples, seed, n_layers, max_degree, set_fraction, doc_set_fraction, preset, doc_alpha,
                                 group_alpha)
        prog_c = snap._prog(prog)
        h = C.c_void_p()
        pc = C.byref(prog_c) if prog_c is not None else None
        if shard is None:
            dv = np.asarray(list(devices) if devices else [device], np.int32)
            _lib.check(L.kg_snapshot_synthetic_on(C.byref(p), pc, _ptr(dv), len(dv), C.byref(h)),
                       "kg_snapshot_synthetic_on")
        else:
            _lib.check(L.kg_snapshot_synthetic_shard(C.byref(p), pc, device, shard[0], shard[1], C.byref(h)),
                       "kg_snapshot_synthetic_shard")
        snap._h = h
        snap.shard = shard
        snap.program = prog
        return snap

    @property
    def handle(self):
        return self._h

    def replicas(self) -> List[int]:
        """Devices of the snapshot's replicas (replica 0 first)."""
        L = _lib.load()
        n = L.kg_snapshot_replicas(self._h, None, 0)
        if n < 0:
            raise _lib.KetoGPUError(_lib.last_error())
        a = np.zeros(max(n, 1), np.int32)
        L.kg_snapshot_replicas(self._h, _ptr(a), n)
        return [int(x) for x in a[:n]]

    def info(self) -> dict:
        a = np.zeros(4, np.uint64)
        _lib.check(_lib.load().kg_snapshot_info(self._h, _ptr(a)), "kg_snapshot_info")
        return {"nodes": int(a[0]), "rows": int(a[1]), "set_edges": int(a[2]), "device_bytes": int(a[3])}

    def materialized(self) -> dict:
        """Rewrite materialisation counts (kg_snapshot_materialized): union nodes, of them new ids,
        check-row entries."""
        a = np.zeros(3, np.uint64)
        _lib.check(_lib.load().kg_snapshot_materialized(self._h, _ptr(a)), "kg_snapshot_materialized")
        return {"union_nodes": int(a[0]), "new_nodes": int(a[1]), "check_rows": int(a[2])}

    def tune(self, key: str, value: int) -> None:
        """Engine knobs (kg_snapshot_tune; keto_amd/csrc/kg_abi.cpp tune_one lists them with their ranges;
        29 since round 6 removed the ones that measured flat): tier chain -- back_wgs, back_edges, stream_ecap,
        stream_wgs, stream_steal, grid_wgs, grid_cap, grid_reserve, grid_ms, grid_ms_words, grid_ms_bytes,
        grid_ms_tg_cap, grid_ms_cap, interp_cap2, max_lanes; expand -- expand_gw, expand_gw_wait_us,
        expand_skip_lds (tests); hash-sharded -- shard_local, shard_force_exchange, shard_max_reruns,
        shard_max_bytes, shard_force_overflow (tests), shard_bucket, shard_vis, shard_heavy, shard_budget,
        shard_back_budget, shard_remote_meta (read at the first binding).  Build-time, from the environment:
        KG_ADJX_ORDER=0 lays adjx out in node order instead of hot-first."""
        _lib.check(_lib.load().kg_snapshot_tune(self._h, key.encode(), int(value)), "kg_snapshot_tune")
        self.__dict__.setdefault("tuned", {})[key] = int(value)  # what the Python drivers need to know

    def synth_ids(self) -> dict:
        a = np.zeros(6, np.uint32)
        _lib.check(_lib.load().kg_synth_ids(self._h, _ptr(a)), "kg_synth_ids")
        return dict(zip(["n_docs", "n_groups", "n_users", "n_folders", "user_obj0", "folder_obj0"], map(int, a)))

    def export(self) -> np.ndarray:
        L = _lib.load()
        n = L.kg_snapshot_export(self._h, None, 0)
        if n < 0:
            raise _lib.KetoGPUError(_lib.last_error())
        out = np.zeros((n, 6), np.uint32)
        got = L.kg_snapshot_export(self._h, _ptr(out), n)
        if got != n:
            raise _lib.KetoGPUError(_lib.last_error())
        return out

    def rows(self, keys: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """GetRelationTuples(ns, obj, rel) for a (n,3) array of keys on the device snapshot
        (kg_snapshot_rows): returns (offsets[n+1], tuples (m,6) uint32), key i's rows in shard order at
        tuples[offsets[i]:offsets[i+1]]."""
        L = _lib.load()
        keys = np.asarray(keys, np.uint32).reshape(-1, 3)
        ks = np.zeros((keys.shape[0], 4), np.uint32)
        ks[:, :3] = keys[:, [0, 1, 2]]
        off = np.zeros(keys.shape[0] + 1, np.uint64)
        n = L.kg_snapshot_rows(self._h, _ptr(ks), keys.shape[0], _ptr(off), None, 0)
        if n < 0:
            raise _lib.KetoGPUError(_lib.last_error())
        out = np.zeros((max(n, 1), 6), np.uint32)
        if n:
            got = L.kg_snapshot_rows(self._h, _ptr(ks), keys.shape[0], _ptr(off), _ptr(out), n)
            if got != n:
                raise _lib.KetoGPUError(_lib.last_error())
        return off.astype(np.int64), out[:n]

    def close(self) -> None:
        if self._h:
            _lib.load().kg_snapshot_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def queries_array(q6: np.ndarray, max_depths) -> np.ndarray:
    """(n,6) tuple ids + per-query max depth -> (n,7) uint32 kg_query rows."""
    q6 = np.asarray(q6, np.uint32).reshape(-1, 6)
    out = np.zeros((q6.shape[0], 7), np.uint32)
    out[:, :6] = q6
    out[:, 6] = np.broadcast_to(np.asarray(max_depths, np.int64), (q6.shape[0],)).astype(np.int32).view(np.uint32)
    return out


class Engine:
    """check.Engine: permission checks against a snapshot."""

    def __init__(self, snapshot: Snapshot, config: Optional[Config] = None):
        self.snapshot = snapshot
        self.config = config or Config()
        self.last_stats: Optional[dict] = None

    # ---- batched (the hot path)
    def batch_check_ids(self, q: np.ndarray, with_stats: bool = False) -> Tuple[np.ndarray, np.ndarray]:
        """q: (n,7) uint32 kg_query rows.  Returns (result u8 [0 not member, 1 member, 2 error], err u32)."""
        q = np.ascontiguousarray(q, np.uint32).reshape(-1, 7)
        n = q.shape[0]
        out = np.zeros(n, np.uint8)
        err = np.zeros(n, np.uint32)
        st = _lib.kg_stats()
        rc = _lib.load().kg_check_batch(self.snapshot.handle, _ptr(q), n, self.config.max_read_depth, _ptr(out),
                                        _ptr(err), C.byref(st) if with_stats else None)
        _lib.check(rc, "kg_check_batch")
        self.last_stats = st.as_dict() if with_stats else None
        return out, err

    def batch_check_packed(self, q: np.ndarray, err_cap: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray, int]:
        """The narrow boundary (kg_check_batch_packed): q (n,7) uint32 kg_query rows are packed to 16 B
        (pack_queries = the header's kg_pack_query), answers come back as bytes and the error codes as
        (index, code) pairs of the KG_ERROR answers only.  Returns (result u8, pairs (k, 2) u32, n_err)."""
        pk = _lib.pack_queries(q)
        n = pk.shape[0]
        cap = n if err_cap is None else int(err_cap)
        out = np.zeros(n, np.uint8)
        idx = np.zeros(max(cap, 1), np.uint32)
        code = np.zeros(max(cap, 1), np.uint32)
        n_err = C.c_size_t(0)
        rc = _lib.load().kg_check_batch_packed(self.snapshot.handle, _ptr(pk), n, self.config.max_read_depth, _ptr(out),
                                               _ptr(idx) if cap else None, _ptr(code) if cap else None, cap,
                                               C.byref(n_err), None)
        _lib.check(rc, "kg_check_batch_packed")
        k = min(cap, int(n_err.value))
        return out, np.stack([idx[:k], code[:k]], axis=1), int(n_err.value)

    def batch_check(self, tuples: Sequence[RelationTuple], max_depths) -> Tuple[List[bool], List[Optional[CheckError]]]:
        """BatchCheck(ctx, []*RelationTuple, maxDepth []int) ([]bool, []error) -- SURVEY.md 8b."""
        it = self.snapshot.interner
        q = queries_array(np.asarray([it.tuple_ids(t) for t in tuples], np.uint32).reshape(-1, 6), max_depths)
        out, err = self.batch_check_ids(q)
        allowed = [bool(o == _lib.KG_IS_MEMBER) for o in out]
        errs = [CheckError(int(e)) if o == _lib.KG_ERROR else None for o, e in zip(out, err)]
        return allowed, errs

    # ---- single-query API of the reference
    def check_relation_tuple(self, t: RelationTuple, rest_depth: int, with_tree: bool = True) -> Result:
        """CheckRelationTuple (engine.go:65-80): membership, error, and for a member the tree of the
        branch that answered it (keto_amd/explain.py)."""
        allowed, errs = self.batch_check([t], [rest_depth])
        if errs[0] is not None:
            return Result(MEMBERSHIP_UNKNOWN, errs[0])
        if not allowed[0]:
            return Result(NOT_MEMBER)
        tree = None
        if with_tree:
            tree = self.check_tree(t, rest_depth)
        return Result(IS_MEMBER, None, tree)

    def check_tree(self, t: RelationTuple, rest_depth: int):
        """The tree of a member check, built inside the library (kg_check_tree: the walk over GPU
        sub-check answers and row reads; keto_amd/explain.py is its CPU-tested restatement)."""
        import ctypes as C
        from .ketoapi import CheckTree, TREE_INTERSECTION
        from .namespace import HIDDEN_TTU_PREFIX
        it = self.snapshot.interner
        L = _lib.load()
        ids = [int(x) for x in it.tuple_ids(t)]
        q = (C.c_uint32 * 7)(*ids, rest_depth & 0xFFFFFFFF)
        hidden = [r for r in range(it.n_relations) if it.rel_name(r).startswith(HIDDEN_TTU_PREFIX)]
        hid = (C.c_uint32 * max(1, len(hidden)))(*hidden)
        n = C.c_size_t(0)
        res, err = C.c_uint8(0), C.c_uint32(0)
        cap = 64
        while True:
            buf = (_lib.kg_check_node * cap)()
            rc = L.kg_check_tree(self.snapshot.handle, q, self.config.max_read_depth, hid, len(hidden), buf, cap,
                                 C.byref(n), C.byref(res), C.byref(err))
            if rc == -3 and n.value > cap:
                cap = n.value
                continue
            _lib.check(rc, "kg_check_tree")
            break
        if res.value != _lib.KG_IS_MEMBER:
            return None
        pos = 0

        def build():
            nonlocal pos
            r = buf[pos]
            pos += 1
            kids = [build() for _ in range(r.n_children)]
            tup = it.relation_tuple((r.t.ns, r.t.obj, r.t.rel, r.t.sns, r.t.sobj, r.t.srel)) if r.has_tuple else None
            typ = _lib.KG_CTREE[r.type]
            return CheckTree(TREE_INTERSECTION if typ == "intersection" else typ, tup, kids)

        return build()

    def check_is_member(self, t: RelationTuple, rest_depth: int) -> bool:
        """CheckIsMember (engine.go:54-60): membership only (no tree)."""
        allowed, errs = self.batch_check([t], [rest_depth])
        if errs[0] is not None:
            raise errs[0]
        return allowed[0]


class ExpandEngine:
    """expand.Engine: subject-set trees."""

    def __init__(self, snapshot: Snapshot, config: Optional[Config] = None):
        self.snapshot = snapshot
        self.config = config or Config()

    def build_trees_ids(self, roots: np.ndarray, device: bool = False) -> List[Optional[np.ndarray]]:
        """roots: (n,4) uint32 kg_set rows (sns, sobj, srel, max_depth).  Returns per root the pre-order
        records (m, 6) = (type, is_set, ns, obj, rel, n_children), or None for a nil tree.  device: through
        kg_expand_batch_device (roots and trees in HBM; the trees are copied back here to be returned)."""
        roots = np.ascontiguousarray(roots, np.uint32).reshape(-1, 4)
        buf = _lib.kg_tree_buf()
        L = _lib.load()
        if device:
            import torch
            dev = torch.device("cuda", self.snapshot.device)
            droots = torch.from_numpy(roots.view(np.int32)).to(dev)
            rc = L.kg_expand_batch_device(self.snapshot.handle, C.c_void_p(droots.data_ptr()), roots.shape[0],
                                          self.config.max_read_depth, C.byref(buf),
                                          C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
            _lib.check(rc, "kg_expand_batch_device")
        else:
            rc = L.kg_expand_batch(self.snapshot.handle, _ptr(roots), roots.shape[0], self.config.max_read_depth,
                                   C.byref(buf))
            _lib.check(rc, "kg_expand_batch")
        try:
            n = int(buf.n_nodes)
            if device:
                recs = np.zeros((n, 5), np.uint32)
                offs = np.zeros(roots.shape[0] + 1, np.uint64)
                _lib.device_to_host(recs, buf.nodes, n * 20)
                _lib.device_to_host(offs, buf.root_off, offs.nbytes)
            else:
                recs = np.ctypeslib.as_array(C.cast(buf.nodes, C.POINTER(C.c_uint32)), shape=(n * 5,)).reshape(n, 5) \
                    if n else np.zeros((0, 5), np.uint32)
                offs = np.ctypeslib.as_array(buf.root_off, shape=(roots.shape[0] + 1,)).copy()
            out: List[Optional[np.ndarray]] = []
            for r in range(roots.shape[0]):
                a, b = int(offs[r]), int(offs[r + 1])
                if a == b:
                    out.append(None)
                    continue
                seg = recs[a:b]
                rec = np.zeros((b - a, 6), np.int64)
                rec[:, 0] = seg[:, 0] & 0xFF
                rec[:, 1] = (seg[:, 0] >> 8) & 0xFF
                rec[:, 2:5] = seg[:, 1:4]
                rec[:, 5] = seg[:, 4]
                out.append(rec)
            return out
        finally:
            L.kg_tree_free(C.byref(buf))

    def build_tree(self, subject, rest_depth: int) -> Optional[Tree]:
        """BuildTree(ctx, subject, restDepth): subject is a SubjectSet or a subject-id string."""
        it = self.snapshot.interner
        if isinstance(subject, SubjectSet):
            row = [*it.subject_set_ids(subject), rest_depth]
        else:
            row = [SUBJECT_ID, it.obj_id(subject), 0, rest_depth]
        row[3] = np.int32(row[3]).view(np.uint32)
        rec = self.build_trees_ids(np.asarray([row], np.uint32))[0]
        return records_to_tree(rec, it)


def records_to_tree(rec: Optional[np.ndarray], it: Interner) -> Optional[Tree]:
    if rec is None or len(rec) == 0:
        return None
    pos = 0

    def walk() -> Tree:
        nonlocal pos
        r = rec[pos]
        pos += 1
        t = Tree(TREE_UNION if int(r[0]) == 1 else TREE_LEAF, it.subject_from_ids(bool(r[1]), int(r[2]), int(r[3]),
                                                                                  int(r[4])))
        for _ in range(int(r[5])):
            t.children.append(walk())
        return t

    return walk()


class Registry:
    """Test/embedding convenience mirroring driver.Registry's engine wiring
    (internal/driver/registry_default.go:180-192): tuples + namespaces -> snapshot + engines."""

    def __init__(self, tuples: Sequence[RelationTuple], namespaces: Sequence[Namespace] = (), max_read_depth: int = 5,
                 device: int = 0, interner: Optional[Interner] = None, devices: Optional[Sequence[int]] = None):
        self.interner = interner or Interner()
        self.config = Config(max_read_depth, list(namespaces))
        self.program = compile_program(list(namespaces), self.interner)
        arr = self.interner.tuples_array(tuples)
        self.snapshot = Snapshot(arr, self.interner, self.program, device, devices=devices)
        self.mapper = Mapper(self.interner, list(namespaces) if namespaces else None)

    def permission_engine(self) -> Engine:
        return Engine(self.snapshot, self.config)

    def expand_engine(self) -> ExpandEngine:
        return ExpandEngine(self.snapshot, self.config)
