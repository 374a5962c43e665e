"""String <-> dense-id interning, the host-side counterpart of the reference ``Mapper``.

The reference maps every object / subject-id string to ``uuid.NewV5(networkID, s)``
(internal/persistence/sql/uuid_mapping.go:31-66) and namespaces are looked up by name
(internal/relationtuple/uuid_mapping.go:180-238, ``FromTuple``).  The engine works on dense u32
ids; one id per UUID is equivalent, so objects and subject ids share ONE id space exactly as
they share the UUID space upstream.  Like ``MapStringsToUUIDs`` (which inserts on read), unknown
strings get a fresh id at query time: a fresh id has no rows, which is what a fresh UUID has.
"""
from __future__ import annotations

import threading
import uuid
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .ketoapi import RelationTuple, SubjectSet

SUBJECT_ID = 0xFFFFFFFF  # KG_SUBJECT_ID
WILDCARD_RELATION = "..."  # internal/check/engine.go:40


class NamespaceNotFound(KeyError):
    """herodot.ErrNotFound from GetNamespaceByName (mapped to ``false`` by REST check,
    internal/check/handler.go:156-160, and to an error by gRPC, :261-264)."""


class Interner:
    def __init__(self, network_id: uuid.UUID = uuid.UUID(int=0)):
        self.network_id = network_id
        self._ns: Dict[str, int] = {}
        self._ns_names: List[str] = []
        self._rel: Dict[str, int] = {}
        self._rel_names: List[str] = []
        self._obj: Dict[str, int] = {}
        self._obj_names: List[str] = []
        # id creation is check-then-insert on three structures: callers on many threads (the request
        # batcher's submitters, the persister's snapshot rebuild) intern concurrently, and two new
        # strings must never share an id -- an unknown subject would then alias a real one
        self._lock = threading.Lock()
        self.rel_id(WILDCARD_RELATION)  # reserve so the wildcard id is stable

    # ---- ids
    def _get(self, d: Dict[str, int], names: List[str], s: str, create: bool, limit: int) -> int:
        v = d.get(s)  # lock-free fast path: an entry, once published, never changes
        if v is not None:
            return v
        if not create:
            raise KeyError(s)
        with self._lock:
            v = d.get(s)
            if v is None:
                v = len(names)
                if v >= limit:
                    raise OverflowError("id space exhausted")
                names.append(s)  # the name first: a reader that sees the id can resolve it
                d[s] = v
        return v

    def ns_id(self, s: str, create: bool = True) -> int:
        return self._get(self._ns, self._ns_names, s, create, 0xFFFF)

    def rel_id(self, s: str, create: bool = True) -> int:
        return self._get(self._rel, self._rel_names, s, create, 0xFFFF)

    def obj_id(self, s: str, create: bool = True) -> int:
        return self._get(self._obj, self._obj_names, s, create, 0x7FFFFFFE)

    def ns_name(self, i: int) -> str:
        return self._ns_names[i]

    def rel_name(self, i: int) -> str:
        return self._rel_names[i]

    def obj_name(self, i: int) -> str:
        return self._obj_names[i]

    def uuid_of(self, s: str) -> uuid.UUID:
        """The reference's internal UUID for a string (uuid_mapping.go:40)."""
        return uuid.uuid5(self.network_id, s)

    @property
    def wildcard_rel(self) -> int:
        return self._rel[WILDCARD_RELATION]

    @property
    def n_namespaces(self) -> int:
        return len(self._ns_names)

    @property
    def n_relations(self) -> int:
        return len(self._rel_names)

    # ---- tuples
    def tuple_ids(self, t: RelationTuple) -> Tuple[int, int, int, int, int, int]:
        ns, obj, rel = self.ns_id(t.namespace), self.obj_id(t.object), self.rel_id(t.relation)
        if t.subject_set is not None:
            s = t.subject_set
            return ns, obj, rel, self.ns_id(s.namespace), self.obj_id(s.object), self.rel_id(s.relation)
        if t.subject_id is None:
            raise ValueError("tuple without subject")
        return ns, obj, rel, SUBJECT_ID, self.obj_id(t.subject_id), 0

    def tuples_array(self, ts: Iterable[RelationTuple]) -> np.ndarray:
        rows = [self.tuple_ids(t) for t in ts]
        return np.asarray(rows, dtype=np.uint32).reshape(-1, 6)

    def relation_tuple(self, ids) -> RelationTuple:
        """The RelationTuple of (ns, obj, rel, sns, sobj, srel) ids (sns == SUBJECT_ID: a subject id)."""
        ns, obj, rel, sns, sobj, srel = (int(x) for x in ids)
        if sns == SUBJECT_ID:
            return RelationTuple(self.ns_name(ns), self.obj_name(obj), self.rel_name(rel), subject_id=self.obj_name(sobj))
        return RelationTuple(self.ns_name(ns), self.obj_name(obj), self.rel_name(rel),
                             subject_set=SubjectSet(self.ns_name(sns), self.obj_name(sobj), self.rel_name(srel)))

    def subject_set_ids(self, s: SubjectSet) -> Tuple[int, int, int]:
        return self.ns_id(s.namespace), self.obj_id(s.object), self.rel_id(s.relation)

    def subject_from_ids(self, is_set: bool, ns: int, obj: int, rel: int):
        if is_set:
            return SubjectSet(self.ns_name(ns), self.obj_name(obj), self.rel_name(rel))
        return self.obj_name(obj)


class Mapper:
    """Namespace-validating mapping (FromTuple / FromSubjectSet, uuid_mapping.go:180-305)."""

    def __init__(self, interner: Interner, namespaces: Optional[Sequence] = None):
        self.interner = interner
        self.namespaces = {n.name for n in namespaces} if namespaces is not None else None

    def _check_ns(self, name: str) -> None:
        if self.namespaces is not None and name not in self.namespaces:
            raise NamespaceNotFound(name)

    def from_tuple(self, t: RelationTuple) -> Tuple[int, int, int, int, int, int]:
        self._check_ns(t.namespace)
        if t.subject_set is not None:
            self._check_ns(t.subject_set.namespace)
        return self.interner.tuple_ids(t)

    def from_subject_set(self, s: SubjectSet) -> Tuple[int, int, int]:
        self._check_ns(s.namespace)
        return self.interner.subject_set_ids(s)
