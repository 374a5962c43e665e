"""The tree of a check result: ``CheckRelationTuple``'s ``Result.Tree``.

The reference builds it while it checks (``internal/check/checkgroup/definitions.go:101-124``
``WithEdge``, ``binop.go:38-69``): a check answered by ``checkDirect`` is a leaf of the request tuple
(``engine.go:165-172``); one answered through a subject-set row is the tree of that row's check
(``engine.go:118-136``: no node of its own); a rewrite child is wrapped in an edge node labelled
with the request tuple and typed by the child (``rewrites.go:59-92,112-139``; an edge over a child
without a tree is a leaf of the request tuple); ``or`` returns its first member child's tree in
child order, ``and`` an ``intersection`` node without tuple over every child's tree, ``not`` keeps
the inner tree and flips the membership (``rewrites.go:141-160``).  ``checkIsAllowed`` runs its
three branches concurrently, so which member branch supplies the tree is schedule-dependent there;
this walk takes direct, then subject-set rows in row order, then the rewrite.

Every membership it relies on is the MI355X engine's: the walk asks ``kg_check_batch`` whether a
sub-check at its rest depth is a member (one batched call per row of candidates) and reads rows
with ``kg_snapshot_rows``.  Only checks at rest depth 0 -- which read no tuple whose answer can
count (``checkDirect`` at depth -1 and every subject-set child at -1 are Unknown) -- are decided
from the rewrite program alone, as ``checkIsAllowed(r, 0)`` does.  Not a hot path: one tree per
call, a handful of small GPU calls per level.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib
from .ketoapi import (CheckTree, RelationTuple, SubjectSet, TREE_COMPUTED, TREE_INTERSECTION, TREE_LEAF, TREE_NOT,
                      TREE_TTU, TREE_UNION)
from .mapper import SUBJECT_ID
from .namespace import HIDDEN_TTU_PREFIX, RW_AND, RW_COMPUTED, RW_NOT, RW_OR, RW_TTU

M, N, E, U = "member", "not_member", "error", "unknown"
Q = Tuple[int, int, int, int, int, int]  # (ns, obj, rel, sns, sobj, srel) ids


class ExplainInconsistent(RuntimeError):
    """The engine said member but no branch reproduces it (never expected)."""


class Explainer:
    """Tree walk for one snapshot and global max depth; memoises rows and sub-check answers."""

    def __init__(self, engine):
        self.engine = engine
        self.snap = engine.snapshot
        self.it = self.snap.interner
        self.wild = self.it.wildcard_rel
        p = self.snap.program
        self.prog = p if p is not None and not p.empty else None
        self.roots: Dict[Tuple[int, int], int] = {}
        if self.prog is not None:
            for ns, rel, root in zip(self.prog.rel_ns, self.prog.rel_rel, self.prog.rel_root):
                self.roots[(int(ns), int(rel))] = int(root)
        self._rows: Dict[Tuple[int, int, int], np.ndarray] = {}
        self._mem: Dict[Tuple[Q, int], Tuple[str, int]] = {}

    # ---- engine access
    def rows(self, ns: int, obj: int, rel: int) -> np.ndarray:
        k = (ns, obj, rel)
        if k not in self._rows:
            _, t = self.snap.rows(np.asarray([k], np.uint32))
            self._rows[k] = t
        return self._rows[k]

    def member(self, qs: List[Q], d: int) -> List[Tuple[str, int]]:
        """checkIsAllowed(q, d) for each q: (M | N | E, error code)."""
        todo = [q for q in dict.fromkeys(qs) if (q, d) not in self._mem]
        if todo:
            if d >= 1:
                from .engine import queries_array
                out, err = self.engine.batch_check_ids(queries_array(np.asarray(todo, np.uint32), d))
                for q, o, e in zip(todo, out, err):
                    self._mem[(q, d)] = (M if o == _lib.KG_IS_MEMBER else E if o == _lib.KG_ERROR else N, int(e))
            else:
                for q in todo:
                    self._mem[(q, d)] = self._depth0(q, ()) if d == 0 else (N, 0)
        return [self._mem[(q, d)] for q in qs]

    # ---- astRelationFor (engine.go:209-229)
    def relation(self, ns: int, rel: int) -> Tuple[str, int]:
        """('none', -1) | ('rewrite', root) | ('error', code)."""
        if self.prog is None or ns >= len(self.prog.ns_has_rel) or not self.prog.ns_has_rel[ns]:
            return "none", -1
        root = self.roots.get((ns, rel))
        if root is None:
            return "error", _lib.KG_ERR_RELATION_NOT_FOUND
        return ("rewrite", root) if root >= 0 else ("none", -1)

    # ---- rest depth 0: only the rewrite program can answer
    def _depth0(self, q: Q, stack) -> Tuple[str, int]:
        kind, root = self.relation(q[0], q[2])
        if kind == "error":
            return E, root
        if kind == "none":
            return N, 0
        if q in stack:
            return E, _lib.KG_ERR_REWRITE_CYCLE
        return self._r0(root, q, stack + (q,))

    def _r0(self, idx: int, q: Q, stack) -> Tuple[str, int]:
        kind, rel, _crel, first, count = (int(x) for x in self.prog.rw[idx])
        if kind in (RW_OR, RW_AND):
            if count == 0:
                return N, 0
            for c in self.prog.child[first:first + count]:
                m, e = self._c0(int(c), q, stack)
                if m == E:
                    return E, e
                if kind == RW_OR and m == M:
                    return M, 0
                if kind == RW_AND and m != M:
                    return N, 0
            return (M, 0) if kind == RW_AND else (N, 0)
        return self._c0(idx, q, stack)

    def _c0(self, idx: int, q: Q, stack) -> Tuple[str, int]:
        kind, rel, _crel, first, _count = (int(x) for x in self.prog.rw[idx])
        if kind == RW_COMPUTED:
            return self._depth0((q[0], q[1], rel) + q[3:], stack)
        if kind == RW_TTU:
            return N, 0  # every candidate is checkIsAllowed(.., -1): Unknown
        if kind == RW_NOT:
            m, e = self._c0(int(self.prog.child[first]), q, stack)
            return (N, 0) if m == M else (M, 0) if m == N else (m, e)
        return self._r0(idx, q, stack)

    # ---- trees (depth >= 1 from here on; depth 0 has no tuple-backed branch)
    def tree(self, q: Q, d: int) -> CheckTree:
        """The tree of checkIsAllowed(q, d), which the engine answered IsMember."""
        if d >= 1:
            if self._direct(q):
                return CheckTree(TREE_LEAF, self.tuple(q))
            kids = self._set_children(q)
            if kids:
                for c, (m, _) in zip(kids, self.member(kids, d - 1)):
                    if m == M:
                        return self.tree(c, d - 1)
        kind, root = self.relation(q[0], q[2])
        if kind == "rewrite":  # at depth 0 the only branch (and it holds only through `not`)
            m, _, t = self._rewrite(root, q, d)
            if m == M:
                return t
        raise ExplainInconsistent(f"{self.tuple(q)} at depth {d}: no member branch")

    def _direct(self, q: Q) -> bool:
        r = self.rows(q[0], q[1], q[2])
        return bool(r.size) and bool(((r[:, 3] == q[3]) & (r[:, 4] == q[4]) &
                                      ((r[:, 5] == q[5]) | (q[3] == SUBJECT_ID))).any())

    def _set_children(self, q: Q) -> List[Q]:
        """checkExpandSubject's candidates: subject-set rows other than `...`, first occurrence."""
        r = self.rows(q[0], q[1], q[2])
        out = []
        for t in r:
            if int(t[3]) != SUBJECT_ID and int(t[5]) != self.wild:
                out.append((int(t[3]), int(t[4]), int(t[5])) + q[3:])
        return list(dict.fromkeys(out))

    def _rewrite(self, idx: int, q: Q, d: int) -> Tuple[str, int, Optional[CheckTree]]:
        """checkSubjectSetRewrite (rewrites.go:30-93) + or / and (binop.go)."""
        if d < 0:
            return U, 0, None
        kind, _rel, _crel, first, count = (int(x) for x in self.prog.rw[idx])
        kids = [int(c) for c in self.prog.child[first:first + count]]
        if not kids:
            return N, 0, None
        if kind == RW_OR:
            for c in kids:
                m, e, t = self._edge(c, q, d)
                if m == E:
                    return E, e, None
                if m == M:
                    return M, 0, t
            return N, 0, None
        if kind == RW_AND:
            trees = []
            for c in kids:
                m, e, t = self._edge(c, q, d)
                if m != M:
                    return (E if m == E else N), e, None
                trees.append(t)
            return M, 0, CheckTree(TREE_INTERSECTION, None, trees)
        return E, _lib.KG_ERR_NOT_IMPLEMENTED, None

    def _edge(self, idx: int, q: Q, d: int) -> Tuple[str, int, Optional[CheckTree]]:
        """One rewrite child behind WithEdge(request tuple, child type)."""
        kind, rel, crel, first, _count = (int(x) for x in self.prog.rw[idx])
        if kind == RW_COMPUTED and self.it.rel_name(rel).startswith(HIDDEN_TTU_PREFIX):
            # a lowered tuple-to-subject-set leaf (namespace.lower_ttu_leaves): the hidden relation holds
            # no tuples, so its only member branch is its TTU -- the reference's tree has that TTU edge
            # right here, without a computed edge in between
            _k, root = self.relation(q[0], rel)
            _kind, _r, _c, f2, _n = (int(x) for x in self.prog.rw[root])
            return self._edge(int(self.prog.child[f2]), q, d)
        if kind == RW_COMPUTED:
            etype = TREE_COMPUTED
            m, e, t = self._computed(rel, q, d)
        elif kind == RW_TTU:
            etype = TREE_TTU
            m, e, t = self._ttu(rel, crel, q, d)
        elif kind == RW_NOT:
            etype = TREE_NOT
            if d < 0:
                m, e, t = U, 0, None
            else:
                m, e, t = self._edge(int(self.prog.child[first]), q, d)
                m = N if m == M else M if m == N else m
        else:
            etype = TREE_UNION if kind == RW_OR else TREE_INTERSECTION
            m, e, t = self._rewrite(idx, q, d)
        me = self.tuple(q)
        return m, e, CheckTree(TREE_LEAF, me) if t is None else CheckTree(etype, me, [t])

    def _computed(self, rel: int, q: Q, d: int):
        if d < 0:
            return U, 0, None
        c = (q[0], q[1], rel) + q[3:]
        m, e = self.member([c], d)[0]
        return m, e, (self.tree(c, d) if m == M else None)

    def _ttu(self, rel: int, crel: int, q: Q, d: int):
        if d < 0:
            return U, 0, None
        r = self.rows(q[0], q[1], rel)
        cands = list(dict.fromkeys((int(t[3]), int(t[4]), crel) + q[3:] for t in r if int(t[3]) != SUBJECT_ID))
        if not cands or d - 1 < 0:
            return N, 0, None
        res = self.member(cands, d - 1)
        for c, (m, _) in zip(cands, res):
            if m == M:
                return M, 0, self.tree(c, d - 1)
        for m, e in res:
            if m == E:
                return E, e, None
        return N, 0, None

    # ---- ids -> API tuples
    def tuple(self, q: Q) -> RelationTuple:
        it = self.it
        ns, obj, rel = it.ns_name(q[0]), it.obj_name(q[1]), it.rel_name(q[2])
        if q[3] == SUBJECT_ID:
            return RelationTuple(ns, obj, rel, subject_id=it.obj_name(q[4]))
        return RelationTuple(ns, obj, rel, subject_set=SubjectSet(it.ns_name(q[3]), it.obj_name(q[4]),
                                                                  it.rel_name(q[5])))
