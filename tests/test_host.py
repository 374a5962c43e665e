"""CPU tests: host logic, tuple codec, namespace compiler, and the C-ABI library surface
(load + exports only; no compute call without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from keto_amd.ketoapi import MalformedInput, RelationTuple, SubjectSet, Tree
from keto_amd.mapper import Interner, Mapper, NamespaceNotFound, SUBJECT_ID
from keto_amd.namespace import (ComputedSubjectSet, InvertResult, Namespace, Relation, SubjectSetRewrite,
                                TupleToSubjectSet, compile_program, namespace_from_json, namespace_to_json)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tuple_string_roundtrip():
    # ketoapi/enc_string.go:13-95
    t = RelationTuple.from_string("doc:readme#editor@(group:dev#member)")
    assert t.subject_set == SubjectSet("group", "dev", "member")
    assert str(t) == "doc:readme#editor@(group:dev#member)"
    t2 = RelationTuple.from_string("doc:folder#parent@doc:folder_c#...")
    assert t2.subject_set == SubjectSet("doc", "folder_c", "...")
    t3 = RelationTuple.from_string("videos:/cats/1.mp4#view@*")
    assert t3.subject_id == "*" and t3.object == "/cats/1.mp4"
    assert RelationTuple.from_string(":directory#access@user").namespace == ""
    for bad in ["nocolon", "ns:obj", "ns:obj#rel"]:
        with pytest.raises(MalformedInput):
            RelationTuple.from_string(bad)


def test_interner_shared_uuid_space():
    it = Interner()
    a = it.tuple_ids(RelationTuple.from_string("n:user#rel@user"))
    assert a[1] == a[4]  # object "user" and subject id "user" share the id (one UUID space)
    assert a[3] == SUBJECT_ID
    assert it.rel_name(it.wildcard_rel) == "..."
    assert it.uuid_of("x") == it.uuid_of("x")


def test_mapper_unknown_namespace():
    it = Interner()
    m = Mapper(it, [Namespace("known")])
    m.from_tuple(RelationTuple.from_string("known:o#r@s"))
    with pytest.raises(NamespaceNotFound):
        m.from_tuple(RelationTuple.from_string("unknown:o#r@s"))
    with pytest.raises(NamespaceNotFound):
        m.from_tuple(RelationTuple.from_string("known:o#r@(unknown:o#r)"))


def test_namespace_json_roundtrip_and_compile():
    js = {"name": "acl", "relations": [
        {"name": "allow"}, {"name": "deny"},
        {"name": "access", "rewrite": {"operator": "and", "children": [
            {"relation": "allow"}, {"inverted": {"relation": "deny"}},
            {"relation": "parent", "computed_subject_set_relation": "access"}]}}]}
    ns = namespace_from_json(js)
    assert isinstance(ns.relations[2].rewrite.children[1], InvertResult)
    assert namespace_from_json(namespace_to_json(ns)) == ns
    it = Interner()
    p = compile_program([ns], it, lower_ttu=False)
    assert p.ns_has_rel[it.ns_id("acl")] == 1
    assert list(p.rel_root) == [-1, -1, 0]
    kinds = list(p.rw[:, 0])
    assert kinds == [1, 2, 4, 2, 3]  # and, computed, not, computed(deny), ttu
    # lowered (the engine's program): the TTU leaf of the `and` becomes computed(hidden), a hidden relation
    # of the same namespace whose rewrite is or(ttu) -- a union the engine materialises
    pl = compile_program([ns], it)
    assert list(pl.rw[:, 0]) == [1, 2, 4, 2, 2, 0, 3]
    hidden = it.rel_id("\x1fttu/parent/access")
    assert int(pl.rw[4, 1]) == hidden and list(pl.rel_rel)[-1] == hidden and list(pl.rel_root)[-1] == 5
    # single child without operator is wrapped into an "or" (ast_definitions.go:59-68)
    ns2 = namespace_from_json({"name": "d", "relations": [{"name": "v", "rewrite": {"relation": "o"}}]})
    assert ns2.relations[0].rewrite.operation == "or"


def test_tree_json_roundtrip():
    t = Tree("union", SubjectSet("a", "b", "c"), [Tree("leaf", "u")])
    assert Tree.from_json(t.to_json()) == t


def test_library_exports_every_declared_symbol():
    from keto_amd import _lib
    from keto_amd.build import build
    build()  # cross-compiles for gfx950 on a CPU-only host too
    with open(os.path.join(ROOT, "include", "ketogpu.h")) as f:
        hdr = f.read()
    # header-only helpers (static inline, e.g. kg_pack_query) are not library symbols
    inline = set(re.findall(r"static inline \w+ (kg_[a-z_]+)\s*\(", hdr))
    declared = set(re.findall(r"\b(kg_[a-z_]+)\s*\(", hdr)) - inline
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    L = _lib.load()
    for name in declared:
        assert hasattr(L, name), name
    assert L.kg_version().startswith(b"ketogpu")


def test_library_reports_errors_without_gpu():
    from keto_amd import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    rc = L.kg_snapshot_create(None, 0, None, None, 0, None)
    assert rc != 0
    assert "NULL" in _lib.last_error()


@pytest.mark.parametrize("seed", range(6))
def test_ttu_lowering_preserves_semantics(seed):
    """namespace.lower_ttu_leaves: the oracle (oracle/keto_oracle.c, rewrites.go restated) gives the same
    answers and errors for the program as written and the lowered one, on random programs with every
    rewrite kind (TTU leaves under and / not / nested or), every depth."""
    import numpy as np
    from test_gpu_check import random_program, random_queries
    from keto_amd.ketoapi import RelationTuple
    from keto_amd.mapper import Interner
    from keto_amd.namespace import compile_program
    from oracle.oracle import POLICY_CANONICAL, Oracle
    rng = np.random.default_rng(3300 + seed)
    nss, rels = ["a", "b", "c"], ["r0", "r1", "r2", "r3"]
    it = Interner()
    namespaces = random_program(rng, nss, rels)
    ref = compile_program(namespaces, it, lower_ttu=False)
    low = compile_program(namespaces, it)
    tuples = []
    for _ in range(200 + 50 * seed):
        ns, obj, rel = rng.choice(nss), f"o{rng.integers(40)}", rng.choice(rels)
        s = f"({rng.choice(nss)}:o{rng.integers(40)}#{rng.choice(rels + ['...'])})" if rng.random() < 0.5 \
            else f"u{rng.integers(20)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    t6 = it.tuples_array(tuples)
    qs = random_queries(rng, nss, rels, 1500, n_obj=40, n_users=20)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(-1, 7, len(qs))
    o1, o2 = Oracle(t6, it.wildcard_rel, ref), Oracle(t6, it.wildcard_rel, low)
    assert len(low.rw) > len(ref.rw) or not any(int(k) == 3 for k in ref.rw[:, 0])
    for gmax in (1, 3, 6):
        e1, r1, _ = o1.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        e2, r2, _ = o2.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        assert (e1 == e2).all() and (r1 == r2).all(), gmax


def test_pack_queries_matches_header(tmp_path):
    """keto_amd._lib.pack_queries (what the tests and bench feed kg_check_batch_packed) equals the header's
    kg_pack_query (what a cgo caller compiles), and a restatement of the device unpack (kg_check.hip
    k_unpack) restores every field -- depths clamped to 0..65535, a subject id's relation ignored."""
    import ctypes as C
    import subprocess
    from keto_amd import _lib
    src = tmp_path / "pack.c"
    src.write_text('#include "ketogpu.h"\n'
                   'int pack_all(const kg_query* q, unsigned long n, kg_query_packed* p) {\n'
                   '  for (unsigned long i = 0; i < n; i++) if (kg_pack_query(q + i, p + i)) return -1;\n'
                   '  return 0; }\n')
    so = tmp_path / "pack.so"
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(so)],
                   check=True)
    lib = C.CDLL(str(so))
    rng = np.random.default_rng(5)
    n = 5000
    q = np.zeros((n, 7), np.uint32)
    q[:, 0] = rng.integers(0, 4095, n)
    q[:, 1] = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    q[:, 2] = rng.integers(0, 4095, n)
    sid = rng.random(n) < 0.5
    q[:, 3] = np.where(sid, 0xFFFFFFFF, rng.integers(0, 4095, n))
    q[:, 4] = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    q[:, 5] = rng.integers(0, 4095, n)
    q[:, 6] = rng.integers(-5, 70000, n).astype(np.int32).view(np.uint32)
    got = _lib.pack_queries(q)
    want = np.zeros((n, 4), np.uint32)
    assert lib.pack_all(q.ctypes.data_as(C.c_void_p), C.c_ulong(n), want.ctypes.data_as(C.c_void_p)) == 0
    assert (got == want).all()
    # the device unpack, restated
    w2, w3 = got[:, 2].astype(np.int64), got[:, 3].astype(np.int64)
    sns = (w2 >> 24) | ((w3 & 0xF) << 8)
    assert ((w2 & 0xFFF) == q[:, 0]).all() and (((w2 >> 12) & 0xFFF) == q[:, 2]).all()
    assert (np.where(sns == 4095, 0xFFFFFFFF, sns) == q[:, 3]).all()
    assert (((w3 >> 4) & 0xFFF)[~sid] == q[~sid, 5]).all() and (((w3 >> 4) & 0xFFF)[sid] == 0).all()
    assert ((w3 >> 16) == np.clip(q[:, 6].view(np.int32), 0, 65535)).all()
    assert (got[:, 0] == q[:, 1]).all() and (got[:, 1] == q[:, 4]).all()
    bad = q[:1].copy()
    bad[0, 0] = 5000
    with pytest.raises(ValueError):
        _lib.pack_queries(bad)


def test_bench_device_packer_matches_pack_queries():
    """bench.py packs the headline's device-resident queries with torch ops (pack_queries_device); they
    must be the header's kg_pack_query rows bit for bit, as keto_amd._lib.pack_queries is (pinned above):
    subject ids and subject sets, depths below 0, inside 1..65535 and above it."""
    import sys
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from keto_amd import _lib
    rng = np.random.default_rng(11)
    n = 20000
    q = np.zeros((n, 7), np.uint32)
    q[:, 0] = rng.integers(0, 4095, n)
    q[:, 1] = rng.integers(0, 2 ** 31 - 1, n)
    q[:, 2] = rng.integers(0, 4095, n)
    sid = rng.random(n) < 0.5
    q[:, 3] = np.where(sid, 0xFFFFFFFF, rng.integers(0, 4095, n))
    q[:, 4] = rng.integers(0, 2 ** 31 - 1, n)
    q[:, 5] = rng.integers(0, 4095, n)
    q[:, 6] = rng.integers(-5, 70000, n).astype(np.int32).view(np.uint32)
    got = bench.pack_queries_device(torch.from_numpy(q.view(np.int32))).numpy().view(np.uint32)
    assert (got == _lib.pack_queries(q)).all()
