"""Check trees (CheckRelationTuple's Result.Tree: kg_check_tree in the library, keto_amd/explain.py its
restatement) on the GPU engine.

* the reference's expected paths (rewrites_test.go:183-205, hasPath :263-288) on its fixture;
* every member answer's tree is a proof: a test-side checker walks it against the tuples and the
  namespace program with the reference's tree rules (leaf = a direct tuple at rest depth >= 1, a
  subject-set hop leaves no node, rewrite children are edge nodes labelled with the request tuple,
  `and` = an intersection without tuple over every child) -- on the golden cases and on random
  programs with every rewrite kind, materialisation on and off;
* the tree walk's membership equals the batch answer and the oracle's.
"""
from collections import defaultdict

import numpy as np
import pytest

from golden_cases import Case, all_cases
from keto_amd.engine import IS_MEMBER, NOT_MEMBER, Config, Engine, Registry
from keto_amd.explain import Explainer
from keto_amd.ketoapi import (RelationTuple, SubjectSet, TREE_COMPUTED, TREE_INTERSECTION, TREE_LEAF, TREE_NOT,
                              TREE_TTU, TREE_UNION)
from keto_amd.namespace import ComputedSubjectSet, InvertResult, SubjectSetRewrite, TupleToSubjectSet
from oracle.oracle import POLICY_CANONICAL, Oracle

pytestmark = pytest.mark.gpu


class Proof:
    """Does a tree justify checkIsAllowed(q, d) = IsMember?  (test-side checker)"""

    def __init__(self, tuples, namespaces):
        self.tuples = {str(t) for t in tuples}
        self.rows = defaultdict(list)
        for t in tuples:
            self.rows[(t.namespace, t.object, t.relation)].append(t.subject_set or t.subject_id)
        self.rw = {(n.name, r.name): r.rewrite for n in namespaces for r in n.relations}
        self.memo = {}

    @staticmethod
    def _with(q, ns, obj, rel):
        return RelationTuple(ns, obj, rel, subject_id=q.subject_id, subject_set=q.subject_set)

    def member(self, t, q, d) -> bool:
        key = (id(t), q, d)
        if key not in self.memo:
            self.memo[key] = False  # a cycle proves nothing
            self.memo[key] = self._member(t, q, d)
        return self.memo[key]

    def _member(self, t, q, d) -> bool:
        if d >= 1 and t.type == TREE_LEAF and t.tuple == q and str(q) in self.tuples:
            return True  # checkDirect
        rw = self.rw.get((q.namespace, q.relation))
        if rw is not None and d >= 0 and self.rewrite(t, rw, q, d):
            return True
        if d >= 1:  # checkExpandSubject: the child's tree stands for the parent
            for s in self.rows[(q.namespace, q.object, q.relation)]:
                if isinstance(s, SubjectSet) and s.relation != "...":
                    if self.member(t, self._with(q, s.namespace, s.object, s.relation), d - 1):
                        return True
        return False

    def rewrite(self, t, rw, q, d) -> bool:
        if rw.operation == "and":
            return (t.type == TREE_INTERSECTION and t.tuple is None and len(t.children) == len(rw.children)
                    and all(self.edge(c, k, q, d) for c, k in zip(t.children, rw.children)))
        return any(self.edge(t, k, q, d) for k in rw.children)

    def edge(self, t, k, q, d) -> bool:
        if t.tuple != q or len(t.children) != 1:
            return False
        c = t.children[0]
        if isinstance(k, ComputedSubjectSet):
            return t.type == TREE_COMPUTED and self.member(c, self._with(q, q.namespace, q.object, k.relation), d)
        if isinstance(k, TupleToSubjectSet):
            return t.type == TREE_TTU and d >= 1 and any(
                self.member(c, self._with(q, s.namespace, s.object, k.computed_subject_set_relation), d - 1)
                for s in self.rows[(q.namespace, q.object, k.relation)] if isinstance(s, SubjectSet))
        if isinstance(k, SubjectSetRewrite):
            return t.type == (TREE_INTERSECTION if k.operation == "and" else TREE_UNION) and self.rewrite(c, k, q, d)
        if isinstance(k, InvertResult):  # the inner result is a non-member: its tree is not a proof
            return t.type == TREE_NOT and c.tuple == q
        return False


def _clamp(d, g):
    return g if d <= 0 or g < d else d


CHECK_CASES = all_cases("checks")


@pytest.mark.parametrize("fn,case", CHECK_CASES, ids=[f"{f}:{c['name']}" for f, c in CHECK_CASES])
def test_golden_check_trees(fn, case):
    c = Case(case)
    reg = Registry(c.tuples, c.namespaces, interner=c.it)
    e = reg.permission_engine()
    proof = Proof(c.tuples, c.namespaces)
    n_paths = 0
    for chk in case["checks"]:
        e.config.max_read_depth = chk["global_max_depth"]
        q = RelationTuple.from_string(chk["tuple"])
        r = e.check_relation_tuple(q, chk["max_depth"])
        assert r.err is None and r.membership == (IS_MEMBER if chk["allowed"] else NOT_MEMBER), chk
        if not chk["allowed"]:
            assert r.tree is None
            continue
        assert r.tree is not None and proof.member(r.tree, q, _clamp(chk["max_depth"], chk["global_max_depth"])), \
            (chk, str(r.tree))
        for p in chk.get("paths", []):
            assert r.tree.has_path(p), (p, str(r.tree))
            n_paths += 1
    if fn == "rewrites_test.json":
        assert n_paths == 3


@pytest.mark.parametrize("mat", [1, 0])
@pytest.mark.parametrize("seed", range(6))
def test_random_check_trees(seed, mat, monkeypatch):
    """Random programs with every rewrite kind (test_gpu_check.random_program) on random graphs:
    every member's tree is a proof; memberships equal the oracle's."""
    from test_gpu_check import random_program, random_queries
    from keto_amd.mapper import Interner
    from keto_amd.namespace import compile_program
    monkeypatch.setenv("KG_MATERIALIZE", str(mat))
    rng = np.random.default_rng(700 + seed)
    nss, rels = ["a", "b", "c"], ["r0", "r1", "r2", "r3"]
    it = Interner()
    namespaces = random_program(rng, nss, rels, unions_only=bool(seed % 2))
    prog = compile_program(namespaces, it, lower_ttu=False)  # the oracle: TTU leaves as written
    n_obj, n_users = 20 + 5 * seed, 15
    tuples = []
    for _ in range(120 + 40 * seed):
        ns, obj, rel = rng.choice(nss), f"o{rng.integers(n_obj)}", rng.choice(rels)
        if rng.random() < 0.5:
            s = f"({rng.choice(nss)}:o{rng.integers(n_obj)}#{rng.choice(rels + ['...'])})"
        else:
            s = f"u{rng.integers(n_users)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    reg = Registry(tuples, namespaces, interner=it)
    qs = random_queries(rng, nss, rels, 1000, n_obj=n_obj, n_users=n_users)
    depths = rng.integers(0, 6, len(qs))
    gmax = 5
    e = Engine(reg.snapshot, Config(gmax))
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, prog)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
    proof = Proof(tuples, namespaces)
    n_member = 0
    # every member (up to 60) and a few others through CheckRelationTuple
    pick = list(np.nonzero((exp == 1) & (oerr == 0))[0][:60]) + list(np.nonzero(exp != 1)[0][:20])
    for i in pick:
        q, d = qs[i], int(depths[i])
        r = e.check_relation_tuple(q, d)
        if oerr[i]:
            assert r.err is not None and r.err.code == oerr[i]
            continue
        assert r.err is None and (r.membership == IS_MEMBER) == bool(exp[i]), (str(q), d)
        if r.membership == IS_MEMBER:
            n_member += 1
            assert proof.member(r.tree, q, _clamp(d, gmax)), (str(q), d, str(r.tree))
            # the library's walk (kg_check_tree, C++) builds exactly the tree of keto_amd/explain.py's
            # restatement over the same GPU answers
            py = Explainer(e).tree(tuple(int(x) for x in it.tuple_ids(q)), _clamp(d, gmax))
            assert r.tree.to_json() == py.to_json(), (str(q), d, str(r.tree), str(py))
        else:
            assert r.tree is None
    assert n_member >= 5, n_member
