"""Namespace configuration and subject-set rewrite AST, and their compiler to the flat
rewrite program consumed by the engine (``kg_rewrite_prog`` in include/ketogpu.h).

Mirrors ``internal/namespace/definitions.go:11-26`` and
``internal/namespace/ast/ast_definitions.go:5-68``.  JSON uses the reference's json tags:
``{"name", "types", "rewrite": {"operator": "or"|"and", "children": [...]}}`` with children
``{"relation"}`` (computed), ``{"relation", "computed_subject_set_relation"}`` (tuple-to-subject-set),
``{"inverted": child}`` and nested ``{"operator", "children"}``.
The reference server never wires the OPL parser in; tests build these
structures programmatically (internal/check/rewrites_test.go:20-86), and so can callers here.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Union

import numpy as np

OP_OR = "or"
OP_AND = "and"

RW_OR, RW_AND, RW_COMPUTED, RW_TTU, RW_NOT = 0, 1, 2, 3, 4


@dataclass
class ComputedSubjectSet:
    relation: str


@dataclass
class TupleToSubjectSet:
    relation: str
    computed_subject_set_relation: str


@dataclass
class InvertResult:
    child: "Child"


@dataclass
class SubjectSetRewrite:
    children: List["Child"] = field(default_factory=list)
    operation: str = OP_OR  # ast.OperatorOr is the zero value


Child = Union[ComputedSubjectSet, TupleToSubjectSet, InvertResult, SubjectSetRewrite]


def as_rewrite(c: Child) -> SubjectSetRewrite:
    """ast_definitions.go:59-68 (AsRewrite wraps a single child into an ``or``)."""
    return c if isinstance(c, SubjectSetRewrite) else SubjectSetRewrite([c])


@dataclass
class RelationType:
    namespace: str
    relation: str = ""


@dataclass
class Relation:
    name: str
    types: List[RelationType] = field(default_factory=list)
    rewrite: Optional[SubjectSetRewrite] = None


@dataclass
class Namespace:
    name: str
    relations: List[Relation] = field(default_factory=list)
    id: int = 0


# ------------------------------------------------------------------------------ JSON
def child_from_json(d: dict) -> Child:
    if "operator" in d or "children" in d:
        return SubjectSetRewrite([child_from_json(c) for c in d.get("children", [])],
                                 _op(d.get("operator", OP_OR)))
    if "inverted" in d:
        return InvertResult(child_from_json(d["inverted"]))
    if "computed_subject_set_relation" in d:
        return TupleToSubjectSet(d["relation"], d["computed_subject_set_relation"])
    if "relation" in d:
        return ComputedSubjectSet(d["relation"])
    raise ValueError(f"unknown rewrite child {d!r}")


def _op(s) -> str:
    if s in (OP_OR, 0, None):
        return OP_OR
    if s in (OP_AND, 1):
        return OP_AND
    raise ValueError(f"unknown operator {s!r}")


def child_to_json(c: Child) -> dict:
    if isinstance(c, SubjectSetRewrite):
        return {"operator": c.operation, "children": [child_to_json(x) for x in c.children]}
    if isinstance(c, InvertResult):
        return {"inverted": child_to_json(c.child)}
    if isinstance(c, TupleToSubjectSet):
        return {"relation": c.relation, "computed_subject_set_relation": c.computed_subject_set_relation}
    return {"relation": c.relation}


def namespace_from_json(d: dict) -> Namespace:
    rels = []
    for r in d.get("relations", []) or []:
        rw = r.get("rewrite")
        rels.append(Relation(r["name"],
                             [RelationType(t.get("namespace", ""), t.get("relation", "")) for t in r.get("types", []) or []],
                             as_rewrite(child_from_json(rw)) if rw else None))
    return Namespace(d.get("name", ""), rels, d.get("id", 0))


def namespace_to_json(n: Namespace) -> dict:
    d: dict = {"name": n.name}
    if n.relations:
        d["relations"] = []
        for r in n.relations:
            rd: dict = {"name": r.name}
            if r.types:
                rd["types"] = [{"namespace": t.namespace, **({"relation": t.relation} if t.relation else {})} for t in r.types]
            if r.rewrite is not None:
                rd["rewrite"] = child_to_json(r.rewrite)
            d["relations"].append(rd)
    return d


# ------------------------------------------------------------------------------ compiler
@dataclass
class Program:
    """Flat arrays for kg_rewrite_prog (and the oracle's ko_set_program)."""
    ns_has_rel: np.ndarray  # uint8 [n_ns]
    rel_ns: np.ndarray      # uint32
    rel_rel: np.ndarray     # uint32
    rel_root: np.ndarray    # int32
    rw: np.ndarray          # int32 [n_rw, 5]  (kind, rel, crel, first, count)
    child: np.ndarray       # int32

    @property
    def empty(self) -> bool:
        return not bool(self.ns_has_rel.any())


HIDDEN_TTU_PREFIX = "\x1fttu/"  # hidden relations of lowered tuple-to-subject-set leaves (no tuple can name one)


def _pure_union(c: Child) -> bool:
    if isinstance(c, SubjectSetRewrite):
        return c.operation == OP_OR and all(_pure_union(x) for x in c.children)
    return isinstance(c, (ComputedSubjectSet, TupleToSubjectSet))


def lower_ttu_leaves(namespaces: List[Namespace]) -> List[Namespace]:
    """Boolean rewrites (and / not, rewrites.go:30-159) whose leaves include tuple-to-subject-sets:
    every such TTU(rel, crel) leaf becomes computed(H) with H a hidden relation of the same namespace
    whose rewrite is ``or(TTU(rel, crel))``.  For any depth d, checkIsAllowed((ns,obj,H), d) =
    checkDirect(H) | checkExpandSubject(H) | TTU at d, and H holds no tuples, so it equals the TTU leaf
    evaluated at d (rewrites.go:167-193 keeps the depth, :205-260 lowers it for the targets) -- but H is
    a union, which kg_augment.hip materialises into plain union nodes, so the formula's leaves are all
    computed and kg_formula.hip splits it into rewrite-free sub-checks (single GPU and hash-sharded)
    instead of the interpreter.  Pure unions are left alone (materialised as they are)."""
    out = []
    for n in namespaces:
        hidden: Dict[str, Relation] = {}

        def lower(c: Child) -> Child:
            if isinstance(c, SubjectSetRewrite):
                return SubjectSetRewrite([lower(x) for x in c.children], c.operation)
            if isinstance(c, InvertResult):
                return InvertResult(lower(c.child))
            if isinstance(c, TupleToSubjectSet):
                name = f"{HIDDEN_TTU_PREFIX}{c.relation}/{c.computed_subject_set_relation}"
                if name not in hidden:
                    hidden[name] = Relation(name, [], SubjectSetRewrite([TupleToSubjectSet(c.relation, c.computed_subject_set_relation)]))
                return ComputedSubjectSet(name)
            return c

        rels = []
        for r in n.relations:
            if r.rewrite is None or _pure_union(r.rewrite):
                rels.append(r)
            else:
                rels.append(Relation(r.name, r.types, lower(r.rewrite)))
        out.append(Namespace(n.name, rels + list(hidden.values()), n.id))
    return out


def compile_program(namespaces: List[Namespace], interner, lower_ttu: bool = True) -> Program:
    """Compile namespace configs into the flat rewrite program.  ``interner`` provides
    ``ns_id(name)`` and ``rel_id(name)`` (see keto_amd.mapper.Interner).  lower_ttu: TTU leaves of
    boolean rewrites become hidden union relations (lower_ttu_leaves; the oracle compiles without it,
    so the parity tests check the lowering's semantics)."""
    if lower_ttu:
        namespaces = lower_ttu_leaves(namespaces)
    rw: List[List[int]] = []
    child: List[int] = []
    rel_ns: List[int] = []
    rel_rel: List[int] = []
    rel_root: List[int] = []
    has: Dict[int, int] = {}

    def emit(c: Child) -> int:
        idx = len(rw)
        rw.append([0, -1, -1, 0, 0])
        if isinstance(c, SubjectSetRewrite):
            kids = [emit(x) for x in c.children]
            rw[idx][0] = RW_AND if c.operation == OP_AND else RW_OR
            rw[idx][3] = len(child)
            rw[idx][4] = len(kids)
            child.extend(kids)
        elif isinstance(c, ComputedSubjectSet):
            rw[idx][0] = RW_COMPUTED
            rw[idx][1] = interner.rel_id(c.relation)
        elif isinstance(c, TupleToSubjectSet):
            rw[idx][0] = RW_TTU
            rw[idx][1] = interner.rel_id(c.relation)
            rw[idx][2] = interner.rel_id(c.computed_subject_set_relation)
        elif isinstance(c, InvertResult):
            k = emit(c.child)
            rw[idx][0] = RW_NOT
            rw[idx][3] = len(child)
            rw[idx][4] = 1
            child.append(k)
        else:
            raise ValueError(f"not implemented: {c!r}")
        return idx

    for n in namespaces:
        nid = interner.ns_id(n.name)
        has[nid] = has.get(nid, 0) | (1 if n.relations else 0)
        for r in n.relations:
            rel_ns.append(nid)
            rel_rel.append(interner.rel_id(r.name))
            rel_root.append(emit(r.rewrite) if r.rewrite is not None else -1)
    n_ns = max([interner.n_namespaces] + [k + 1 for k in has])
    ns_has = np.zeros(n_ns, np.uint8)
    for k, v in has.items():
        ns_has[k] = v
    return Program(ns_has,
                   np.asarray(rel_ns, np.uint32), np.asarray(rel_rel, np.uint32), np.asarray(rel_root, np.int32),
                   np.asarray(rw, np.int32).reshape(-1, 5), np.asarray(child, np.int32))
