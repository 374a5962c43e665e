"""CPU tests of the check-tree walk (keto_amd/explain.py) with the engine's two calls answered by the
test oracle (sub-check memberships) and the tuple list (rows): the walk's rules against the
reference's expected paths and the proof checker of tests/test_gpu_explain.py.  The GPU tests run
the same walk on the HIP engine."""
import numpy as np
import pytest

from golden_cases import Case, all_cases
from keto_amd.explain import Explainer
from keto_amd.ketoapi import RelationTuple
from keto_amd.mapper import SUBJECT_ID
from oracle.oracle import POLICY_CANONICAL, Oracle


class _Snap:
    def __init__(self, it, prog, rows6):
        self.interner, self.program, self.t6 = it, prog, rows6

    def rows(self, keys):
        keys = np.asarray(keys, np.uint32).reshape(-1, 3)
        parts = [self.t6[(self.t6[:, 0] == k[0]) & (self.t6[:, 1] == k[1]) & (self.t6[:, 2] == k[2])] for k in keys]
        off = np.concatenate([[0], np.cumsum([len(p) for p in parts])]).astype(np.int64)
        return off, (np.concatenate(parts) if parts else np.zeros((0, 6), np.uint32))


class _Engine:
    """batch_check_ids answered by the oracle (test stand-in for the HIP engine)."""

    def __init__(self, snap, gmax):
        self.snapshot, self.gmax = snap, gmax
        self.oracle = Oracle(snap.t6, snap.interner.wildcard_rel, snap.program)

    def batch_check_ids(self, q):
        q = np.asarray(q, np.uint32).reshape(-1, 7)
        res, err, _ = self.oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), self.gmax, POLICY_CANONICAL)
        out = np.where(err != 0, 2, res).astype(np.uint8)
        return out, err.astype(np.uint32)


def _tree(c, q, d, g):
    snap = _Snap(c.it, c.prog, c.arr)
    d = g if d <= 0 or g < d else d
    return Explainer(_Engine(snap, g)).tree(tuple(int(x) for x in c.it.tuple_ids(q)), d)


def test_rewrites_expected_paths():
    from test_gpu_explain import Proof
    fn, case = [x for x in all_cases("checks") if x[0] == "rewrites_test.json"][0]
    c = Case(case)
    proof = Proof(c.tuples, c.namespaces)
    n = 0
    for chk in case["checks"]:
        if not chk["allowed"]:
            continue
        q = RelationTuple.from_string(chk["tuple"])
        t = _tree(c, q, chk["max_depth"], chk["global_max_depth"])
        assert proof.member(t, q, min(chk["max_depth"], chk["global_max_depth"])), (chk, str(t))
        for p in chk.get("paths", []):
            assert t.has_path(p), (p, str(t))
            n += 1
    assert n == 3


def test_tree_shapes():
    """The reference's shapes: an `and` root without tuple, edges labelled with the request tuple,
    a subject-set hop without a node, `not` over a leaf of the request tuple."""
    fn, case = [x for x in all_cases("checks") if x[0] == "rewrites_test.json"][0]
    c = Case(case)
    t = _tree(c, RelationTuple.from_string("acl:document#access@alice"), 100, 5)
    assert t.type == "intersection" and t.tuple is None and [x.type for x in t.children] == \
        ["computed_subject_set", "not"]
    assert t.children[1].children[0].type == "leaf" and str(t.children[1].children[0].tuple) == \
        "acl:document#access@alice"
    t = _tree(c, RelationTuple.from_string("doc:file#viewer@user"), 100, 5)
    assert t.type == "tuple_to_subject_set" and str(t.tuple) == "doc:file#viewer@user"
    assert "doc:folder_a#owner@user" in str(t)
    # owner@group:editors#... is skipped as a `...` subject set; the TTU over owner reaches member
    t = _tree(c, RelationTuple.from_string("resource:topsecret#owner@mark"), 100, 5)
    assert t.type == "tuple_to_subject_set" and t.children[0].type == "leaf"


@pytest.mark.parametrize("seed", range(6))
def test_random_trees(seed):
    """Random programs with every rewrite kind: every member's tree is a proof."""
    from test_gpu_check import random_program, random_queries
    from test_gpu_explain import Proof
    from keto_amd.mapper import Interner
    from keto_amd.namespace import compile_program
    rng = np.random.default_rng(700 + seed)
    nss, rels = ["a", "b", "c"], ["r0", "r1", "r2", "r3"]
    it = Interner()
    namespaces = random_program(rng, nss, rels, unions_only=bool(seed % 2))
    prog = compile_program(namespaces, it)
    n_obj, n_users = 20 + 5 * seed, 15
    tuples = []
    for _ in range(120 + 40 * seed):
        ns, obj, rel = rng.choice(nss), f"o{rng.integers(n_obj)}", rng.choice(rels)
        if rng.random() < 0.5:
            s = f"({rng.choice(nss)}:o{rng.integers(n_obj)}#{rng.choice(rels + ['...'])})"
        else:
            s = f"u{rng.integers(n_users)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    qs = random_queries(rng, nss, rels, 1000, n_obj=n_obj, n_users=n_users)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    snap = _Snap(it, prog, it.tuples_array(tuples))
    gmax = 5
    eng = _Engine(snap, gmax)
    depths = rng.integers(0, 6, len(qs))
    out, err = eng.batch_check_ids(np.concatenate([q6, depths[:, None].astype(np.int32).view(np.uint32)], 1))
    proof = Proof(tuples, namespaces)
    n = 0
    for i, (q, d) in enumerate(zip(qs, depths)):
        if out[i] != 1:
            continue
        dd = gmax if d <= 0 or gmax < d else int(d)
        t = Explainer(eng).tree(tuple(int(x) for x in q6[i]), dd)
        assert proof.member(t, q, dd), (str(q), dd, str(t))
        n += 1
    assert n >= 5, n
