"""Public API types of the check/expand path, mirroring the reference's ``ketoapi`` package.

* ``RelationTuple.from_string`` / ``__str__`` follow ``ketoapi/enc_string.go:13-95``
  (``ns:obj#rel@subject``; a subject containing ``#`` is a subject set, optional parentheses).
* ``Tree`` follows ``ketoapi/public_api_definitions.go:136-183`` (``TreeNodeType`` strings and
  the ``{type, tuple, children}`` JSON shape used by the expand API and its golden outputs).
* ``CheckTree`` is ``Tree[*RelationTuple]`` as a check result carries it
  (``internal/check/checkgroup/definitions.go:46-50``): nodes labelled by whole tuples, ``Label`` /
  ``String`` as ``ketoapi/enc_string.go:101-152``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

TREE_UNION = "union"
TREE_EXCLUSION = "exclusion"
TREE_INTERSECTION = "intersection"
TREE_LEAF = "leaf"
TREE_TTU = "tuple_to_subject_set"
TREE_COMPUTED = "computed_subject_set"
TREE_NOT = "not"
TREE_UNSPECIFIED = "unspecified"


class MalformedInput(ValueError):
    """ketoapi.ErrMalformedInput (enc_string.go:11)."""


@dataclass(frozen=True)
class SubjectSet:
    namespace: str
    object: str
    relation: str

    def __str__(self) -> str:
        return f"{self.namespace}:{self.object}#{self.relation}"

    @staticmethod
    def from_string(s: str) -> "SubjectSet":
        ns_obj, sep, rel = s.partition("#")
        if not sep:
            raise MalformedInput("expected subject set to contain '#'")
        ns, sep, obj = ns_obj.partition(":")
        if not sep:
            raise MalformedInput("expected subject set to contain ':'")
        return SubjectSet(ns, obj, rel)


@dataclass(frozen=True)
class RelationTuple:
    namespace: str
    object: str
    relation: str
    subject_id: Optional[str] = None
    subject_set: Optional[SubjectSet] = None

    def __str__(self) -> str:
        if self.subject_id is not None:
            sub = self.subject_id
        elif self.subject_set is not None:
            sub = f"({self.subject_set})"
        else:
            sub = "<ERROR: no subject>"
        return f"{self.namespace}:{self.object}#{self.relation}@{sub}"

    @staticmethod
    def from_string(s: str) -> "RelationTuple":
        ns, sep, rest = s.partition(":")
        if not sep:
            raise MalformedInput("expected input to contain ':'")
        obj, sep, rest = rest.partition("#")
        if not sep:
            raise MalformedInput("expected input to contain '#'")
        rel, sep, sub = rest.partition("@")
        if not sep:
            raise MalformedInput("expected input to contain '@'")
        sub = sub.strip("()")
        if "#" in sub:
            return RelationTuple(ns, obj, rel, subject_set=SubjectSet.from_string(sub))
        return RelationTuple(ns, obj, rel, subject_id=sub)

    def to_json(self) -> dict:
        d = {"namespace": self.namespace, "object": self.object, "relation": self.relation}
        if self.subject_id is not None:
            d["subject_id"] = self.subject_id
        if self.subject_set is not None:
            d["subject_set"] = {"namespace": self.subject_set.namespace,
                                "object": self.subject_set.object,
                                "relation": self.subject_set.relation}
        return d

    @staticmethod
    def from_json(d: dict) -> "RelationTuple":
        ss = d.get("subject_set")
        return RelationTuple(d.get("namespace", ""), d.get("object", ""), d.get("relation", ""),
                             subject_id=d.get("subject_id"),
                             subject_set=SubjectSet(ss.get("namespace", ""), ss.get("object", ""),
                                                    ss.get("relation", "")) if ss else None)


@dataclass
class Tree:
    """Expand tree node.  ``subject`` is a ``SubjectSet`` or a subject-id string."""
    type: str
    subject: object
    children: List["Tree"] = field(default_factory=list)

    def to_json(self) -> dict:
        """The REST/CLI JSON shape of expand/handler.go (see the docs golden expected_output.json)."""
        t = {"namespace": "", "object": "", "relation": ""}
        if isinstance(self.subject, SubjectSet):
            t["subject_set"] = {"namespace": self.subject.namespace, "object": self.subject.object,
                                "relation": self.subject.relation}
        else:
            t["subject_id"] = self.subject
        d = {"tuple": t, "type": self.type}
        if self.children:
            d["children"] = [c.to_json() for c in self.children]
        return d

    @staticmethod
    def from_json(d: dict) -> "Tree":
        t = d.get("tuple", {})
        if "subject_set" in t and t["subject_set"] is not None:
            s = t["subject_set"]
            subj: object = SubjectSet(s.get("namespace", ""), s.get("object", ""), s.get("relation", ""))
        else:
            subj = t.get("subject_id")
        return Tree(d["type"], subj, [Tree.from_json(c) for c in d.get("children", []) or []])


def trees_equal_unordered(a: Optional[Tree], b: Optional[Tree]) -> bool:
    """Order-insensitive tree equality, as expand.AssertInternalTreesAreEqual
    (internal/expand/testhelper.go:52-76)."""
    if a is None or b is None:
        return a is None and b is None
    if a.type != b.type or a.subject != b.subject or len(a.children) != len(b.children):
        return False
    used = [False] * len(b.children)
    for ca in a.children:
        for j, cb in enumerate(b.children):
            if not used[j] and trees_equal_unordered(ca, cb):
                used[j] = True
                break
        else:
            return False
    return True


@dataclass
class CheckTree:
    """A check result's tree (checkgroup.Result.Tree): ``tuple`` is None for an ``and`` node
    (binop.go:47-50 builds it without one)."""
    type: str
    tuple: Optional[RelationTuple]
    children: List["CheckTree"] = field(default_factory=list)

    def label(self) -> str:
        """Tree.Label (enc_string.go:101-107)."""
        return "" if self.tuple is None else str(self.tuple)

    def __str__(self) -> str:
        """Tree.String (enc_string.go:109-152)."""
        if self.type == TREE_LEAF:
            return f"\u220b {self.label()}\ufe0f"
        kids = []
        for i, c in enumerate(self.children):
            indent = "   " if i == len(self.children) - 1 else "\u2502  "
            kids.append(("\n" + indent).join(str(c).split("\n")))
        op = {TREE_INTERSECTION: "and", TREE_UNION: "or", TREE_EXCLUSION: "\\", TREE_NOT: "not",
              TREE_TTU: "\u2510 tuple to userset", TREE_COMPUTED: "\u2510 computed userset"}.get(self.type, "")
        box = "\u2514" if len(kids) == 1 else "\u251c"
        return f"{op} {self.label()}\n{box}\u2500\u2500" + "\n\u2514\u2500\u2500".join(kids)

    def to_json(self) -> dict:
        d: dict = {"type": self.type}
        if self.tuple is not None:
            d["tuple"] = self.tuple.to_json()
        if self.children:
            d["children"] = [c.to_json() for c in self.children]
        return d

    def has_path(self, path: List[str]) -> bool:
        """rewrites_test.go:263-288 (hasPath): labels from this node down one branch, "*" matches any."""
        if not path:
            return True
        if path[0] != "*" and path[0] != self.label():
            return False
        return len(path) == 1 or any(c.has_path(path[1:]) for c in self.children)
