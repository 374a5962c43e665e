"""GPU snapshot persister: the reference's ``relationtuple.Manager`` over an HBM snapshot
(SURVEY.md §8f rank 3).

Reference behaviour mirrored (paths relative to the reference checkout):
  Manager interface (Get / Write / Delete / DeleteAll / Transact)   internal/relationtuple/definitions.go:19-25
  GetRelationTuples: filter, ORDER BY shard_id, keyset page         internal/persistence/sql/relationtuples.go:203-244
    (``shard_id > lastID``, LIMIT per_page+1, next token = the last returned row's shard id)
  page size default 100, token = shard-id UUID string, bad token    internal/persistence/sql/persister.go:24-38,97-125
    -> ErrMalformedPageToken
  InsertRelationTuple: fresh UUIDv4 shard id per row, nil subject   relationtuples.go:100-122
    -> ErrNilSubject; no uniqueness constraint (duplicates kept)
  DeleteRelationTuples: every row equal to the tuple, in one tx     relationtuples.go:164-185
  DeleteAllRelationTuples: every row matching the query             relationtuples.go:187-201
  TransactRelationTuples: writes then deletes, all-or-nothing       relationtuples.go:260-270
  whereSubject: a subject-id query matches only subject-id rows,    relationtuples.go:124-145
    a subject-set query only subject-set rows

The rows live on the host in shard order (the source of truth, like the SQL table); the check /
expand engines read an immutable GPU snapshot built from them.  Every successful write bumps a
version; the next engine call after a write rebuilds the snapshot (``kg_snapshot_create``) from
the rows in shard order, so a check always sees every committed write (read-your-writes).  Reads
of the tuple list (``get_relation_tuples``) are not on the hot path and are answered from the
host rows.  Shard ids come from a seeded generator so runs are reproducible (the reference draws
them from crypto/rand; only their order matters, and no reference test pins it).
"""
from __future__ import annotations

import random
import threading
import uuid
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

from .engine import Config, Engine, ExpandEngine, Snapshot
from .ketoapi import RelationTuple, SubjectSet
from .mapper import Interner, Mapper
from .namespace import Namespace, compile_program

DEFAULT_PAGE_SIZE = 100  # persister.go:38


class NilSubject(ValueError):
    """ketoapi.ErrNilSubject."""


class MalformedPageToken(ValueError):
    """persistence.ErrMalformedPageToken."""


@dataclass(frozen=True)
class RelationQuery:
    """relationtuple.RelationQuery: every field is optional; ``subject_id`` and ``subject_set``
    are mutually exclusive (one Subject)."""
    namespace: Optional[str] = None
    object: Optional[str] = None
    relation: Optional[str] = None
    subject_id: Optional[str] = None
    subject_set: Optional[SubjectSet] = None

    def matches(self, t: RelationTuple) -> bool:
        if self.namespace is not None and t.namespace != self.namespace:
            return False
        if self.object is not None and t.object != self.object:
            return False
        if self.relation is not None and t.relation != self.relation:
            return False
        if self.subject_id is not None:  # whereSubject, SubjectID branch: subject-set columns NULL
            return t.subject_set is None and t.subject_id == self.subject_id
        if self.subject_set is not None:  # SubjectSet branch: subject_id NULL
            return t.subject_id is None and t.subject_set == self.subject_set
        return True


def _check_subject(t: RelationTuple) -> None:
    if t.subject_id is None and t.subject_set is None:
        raise NilSubject("subject is not allowed to be nil")


class SnapshotPersister:
    """relationtuple.Manager whose reads for check / expand come from a GPU snapshot."""

    def __init__(self, namespaces: Sequence[Namespace] = (), max_read_depth: int = 5, device: int = 0,
                 seed: int = 0, interner: Optional[Interner] = None, devices: Optional[Sequence[int]] = None):
        self.interner = interner or Interner()
        self.namespaces = list(namespaces)
        self.config = Config(max_read_depth, self.namespaces)
        self.program = compile_program(self.namespaces, self.interner)
        self.mapper = Mapper(self.interner, self.namespaces if self.namespaces else None)
        self.device = device
        self.devices = list(devices) if devices else None  # replicas (kg_snapshot_create_on)
        self._rng = random.Random(seed)
        self._rows: List[Tuple[uuid.UUID, RelationTuple]] = []  # sorted by shard id
        self._lock = threading.RLock()
        self._version = 0
        self._snap: Optional[Snapshot] = None
        self._snap_version = -1
        self.rebuilds = 0

    # ---- writes (each one is a transaction: validate everything, then apply)
    def _shard_id(self) -> uuid.UUID:
        return uuid.UUID(int=self._rng.getrandbits(128), version=4)

    def _apply(self, ins: Sequence[RelationTuple], dels: Sequence[RelationTuple]) -> None:
        for t in list(ins) + list(dels):
            _check_subject(t)
        if not ins and not dels:
            return
        rows = list(self._rows)
        for t in ins:
            rows.append((self._shard_id(), t))
        if dels:
            gone = set(dels)
            rows = [r for r in rows if r[1] not in gone]
        rows.sort(key=lambda r: r[0].int)
        self._rows = rows
        self._version += 1

    def write_relation_tuples(self, *ts: RelationTuple) -> None:
        with self._lock:
            self._apply(ts, ())

    def delete_relation_tuples(self, *ts: RelationTuple) -> None:
        with self._lock:
            self._apply((), ts)

    def transact_relation_tuples(self, ins: Sequence[RelationTuple], dels: Sequence[RelationTuple]) -> None:
        with self._lock:
            self._apply(ins, dels)

    def delete_all_relation_tuples(self, query: RelationQuery) -> None:
        with self._lock:
            rows = [r for r in self._rows if not query.matches(r[1])]
            if len(rows) != len(self._rows):
                self._rows = rows
                self._version += 1

    # ---- reads of the tuple list
    def get_relation_tuples(self, query: RelationQuery, page_token: str = "",
                            page_size: int = 0) -> Tuple[List[RelationTuple], str]:
        per_page = page_size or DEFAULT_PAGE_SIZE
        if page_token:
            try:
                last = uuid.UUID(page_token).int
            except ValueError as e:
                raise MalformedPageToken(page_token) from e
        else:
            last = 0  # uuid.Nil
        with self._lock:
            rows = self._rows
        res: List[Tuple[uuid.UUID, RelationTuple]] = []
        for sid, t in rows:
            if sid.int > last and query.matches(t):
                res.append((sid, t))
                if len(res) > per_page:
                    break
        token = ""
        if len(res) > per_page:
            res = res[:per_page]
            token = str(res[-1][0])
        return [t for _, t in res], token

    def __len__(self) -> int:
        return len(self._rows)

    # ---- the GPU snapshot the engines read
    @property
    def version(self) -> int:
        return self._version

    def snapshot(self) -> Snapshot:
        """The snapshot of the current rows; rebuilt on the first call after a write."""
        with self._lock:
            if self._snap is None or self._snap_version != self._version:
                arr = self.interner.tuples_array(t for _, t in self._rows)
                snap = Snapshot(arr, self.interner, self.program, self.device, devices=self.devices)
                self._snap, self._snap_version = snap, self._version
                self.rebuilds += 1
            return self._snap

    def permission_engine(self) -> Engine:
        return _LiveEngine(self)

    def expand_engine(self) -> ExpandEngine:
        return _LiveExpandEngine(self)


class _LiveEngine(Engine):
    """check.Engine bound to a persister: every batch reads the persister's current snapshot and
    holds a reference to it for the duration of the call (a concurrent write only swaps the
    persister's pointer; the replaced snapshot is destroyed when its last reader lets go)."""

    def __init__(self, p: SnapshotPersister):
        self._p = p
        super().__init__(None, p.config)

    @property
    def snapshot(self) -> Snapshot:
        return self._p.snapshot()

    @snapshot.setter
    def snapshot(self, _v) -> None:
        pass

    @property
    def interner(self) -> Interner:
        return self._p.interner

    def batch_check_ids(self, q, with_stats: bool = False):
        e = Engine(self._p.snapshot(), self.config)
        try:
            return e.batch_check_ids(q, with_stats)
        finally:
            self.last_stats = e.last_stats


class _LiveExpandEngine(ExpandEngine):
    def __init__(self, p: SnapshotPersister):
        self._p = p
        super().__init__(None, p.config)

    @property
    def snapshot(self) -> Snapshot:
        return self._p.snapshot()

    @snapshot.setter
    def snapshot(self, _v) -> None:
        pass

    def build_trees_ids(self, roots):
        return ExpandEngine(self._p.snapshot(), self.config).build_trees_ids(roots)
