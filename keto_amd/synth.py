"""Synthetic Drive-like tuple graphs generated in HBM.

The generator itself is device code (keto_amd/csrc/kg_synth.h); this module supplies the id
scheme it assumes and, for preset C3, the OPL namespace program:

    doc / folder:  view  = viewer | edit | parents.traverse(view)
                   edit  = editor | owner | parents.traverse(edit)
    doc:           share = view & !blocked
"""
from __future__ import annotations

from typing import List

import numpy as np

from .mapper import Interner
from .namespace import (ComputedSubjectSet, InvertResult, Namespace, Relation, SubjectSetRewrite,
                        TupleToSubjectSet, compile_program)

PRESET_C2 = 0
PRESET_C3 = 1

NAMESPACES = ["doc", "group", "user", "folder"]
RELATIONS = ["viewer", "member", "editor", "owner", "parents", "blocked", "view", "edit", "share"]  # after "..."


# Config C3's namespaces in OPL (keto_amd.opl parses this into exactly c3_namespaces(); the tests
# check that both compile to the same rewrite program).
C3_OPL = """
class user implements Namespace {}

class doc implements Namespace {
  related: {
    viewer: (user | SubjectSet<group, "member">)[]
    editor: (user | SubjectSet<group, "member">)[]
    owner: user[]
    parents: folder[]
    blocked: user[]
  }
  permits = {
    view: (ctx: Context): boolean =>
      this.related.viewer.includes(ctx.subject) ||
      this.related.edit.includes(ctx.subject) ||
      this.related.parents.traverse(p => p.permits.view(ctx)),
    edit: (ctx: Context): boolean =>
      this.related.editor.includes(ctx.subject) ||
      this.related.owner.includes(ctx.subject) ||
      this.related.parents.traverse(p => p.permits.edit(ctx)),
    share: (ctx: Context): boolean =>
      this.related.view.includes(ctx.subject) && !this.related.blocked.includes(ctx.subject),
  }
}

class group implements Namespace {
  related: {
    member: (user | SubjectSet<group, "member">)[]
  }
}

class folder implements Namespace {
  related: {
    viewer: (user | SubjectSet<group, "member">)[]
    editor: (user | SubjectSet<group, "member">)[]
    owner: user[]
    parents: folder[]
  }
  permits = {
    view: (ctx: Context): boolean =>
      this.related.viewer.includes(ctx.subject) ||
      this.related.edit.includes(ctx.subject) ||
      this.related.parents.traverse(p => p.permits.view(ctx)),
    edit: (ctx: Context): boolean =>
      this.related.editor.includes(ctx.subject) ||
      this.related.owner.includes(ctx.subject) ||
      this.related.parents.traverse(p => p.permits.edit(ctx)),
  }
}
"""


def interner() -> Interner:
    it = Interner()  # rel 0 = "..."
    for n in NAMESPACES:
        it.ns_id(n)
    for r in RELATIONS:
        it.rel_id(r)
    return it


def c3_namespaces() -> List[Namespace]:
    def view():
        return SubjectSetRewrite([ComputedSubjectSet("viewer"), ComputedSubjectSet("edit"),
                                  TupleToSubjectSet("parents", "view")])

    def edit():
        return SubjectSetRewrite([ComputedSubjectSet("editor"), ComputedSubjectSet("owner"),
                                  TupleToSubjectSet("parents", "edit")])

    plain = [Relation(r) for r in ("viewer", "editor", "owner", "parents")]
    doc = Namespace("doc", plain + [Relation("blocked"), Relation("view", rewrite=view()),
                                    Relation("edit", rewrite=edit()),
                                    Relation("share", rewrite=SubjectSetRewrite(
                                        [ComputedSubjectSet("view"), InvertResult(ComputedSubjectSet("blocked"))],
                                        "and"))])
    folder = Namespace("folder", [Relation(r) for r in ("viewer", "editor", "owner", "parents")] +
                       [Relation("view", rewrite=view()), Relation("edit", rewrite=edit())])
    group = Namespace("group", [Relation("member")])
    return [doc, group, folder]


def program(preset: int, it: Interner):
    """The namespace program of a preset: C3's comes from its OPL text (keto_amd.opl)."""
    if preset == PRESET_C3:
        from .opl import parse_strict
        return compile_program(parse_strict(C3_OPL), it)
    return None


def hot_group_roots(ids: dict, n: int, max_depth: int = 0) -> np.ndarray:
    """Config C5's expand roots: the n most popular group#member sets of the generator (popularity
    rank r of layer r % 8 -> group by the generator's permutation, keto_amd/csrc/kg_synth.h), as
    (n, 4) uint32 kg_set rows (ns group, object, rel member, request max depth; 0 = global)."""
    n_docs, n_groups = ids["n_docs"], ids["n_groups"]
    gpl = n_groups // 8
    r = np.arange(n, dtype=np.uint64)
    layer, rank = r % 8, r // 8
    node = n_docs + layer * gpl + (rank * 2654435761 + 12345) % gpl
    roots = np.zeros((n, 4), np.uint32)
    roots[:, 0] = NAMESPACES.index("group")
    roots[:, 1] = node.astype(np.uint32)  # group object id == node id
    roots[:, 2] = 1 + RELATIONS.index("member")
    roots[:, 3] = np.uint32(max_depth)
    return roots
