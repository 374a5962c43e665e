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

The rows live on the host in shard order (the source of truth, like the SQL table: a sorted list
keyed by shard id plus a tuple -> shard ids index, so a write costs O(delta log n)); the check /
expand engines read an immutable GPU snapshot built from them.  Every successful write bumps a
version and joins a pending delta; the next engine call after writes refreshes the snapshot
INCREMENTALLY (``kg_snapshot_apply``: only the delta is interned on the host, rows and every
derived structure are rebuilt on the device, inserted rows placed by shard id), so a check always
sees every committed write (read-your-writes).  The first snapshot, and any delta larger than
``rebuild_fraction`` of the rows, is a full ``kg_snapshot_create_ordered``.  Reads of the tuple
list (``get_relation_tuples``) are not on the hot path and are answered from the host rows.  Shard
ids come from a seeded generator so runs are reproducible (the reference draws them from
crypto/rand; only their order matters, and no reference test pins it).
"""
from __future__ import annotations

import random
import threading
import uuid
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
from sortedcontainers import SortedKeyList

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
                 seed: int = 0, interner: Optional[Interner] = None, devices: Optional[Sequence[int]] = None,
                 rebuild_fraction: float = 0.125):
        self.interner = interner or Interner()
        self.namespaces = list(namespaces)
        self.config = Config(max_read_depth, self.namespaces)
        self.program = compile_program(self.namespaces, self.interner)
        self.mapper = Mapper(self.interner, self.namespaces if self.namespaces else None)
        self.device = device
        self.devices = list(devices) if devices else None  # replicas (kg_snapshot_create_on)
        self._rng = random.Random(seed)
        self._rows = SortedKeyList(key=lambda r: r[0].int)  # (shard id, tuple), sorted by shard id
        self._by_tuple: Dict[RelationTuple, List[uuid.UUID]] = {}
        self._lock = threading.RLock()
        self._version = 0
        self._snap: Optional[Snapshot] = None
        self._snap_version = -1
        # the delta since the snapshot: inserted rows (shard id -> tuple), deleted tuple values
        self._p_ins: Dict[int, RelationTuple] = {}
        self._p_del: set = set()
        self.rebuild_fraction = rebuild_fraction
        self.rebuilds = 0  # full builds
        self.applies = 0   # incremental refreshes

    # ---- writes (each one is a transaction: validate everything, then apply)
    def _shard_id(self) -> uuid.UUID:
        return uuid.UUID(int=self._rng.getrandbits(128), version=4)

    def _remove_tuple(self, t: RelationTuple) -> None:
        for sid in self._by_tuple.pop(t, ()):
            self._rows.remove((sid, t))
            self._p_ins.pop(sid.int, None)
        self._p_del.add(t)  # base rows equal to t go too (relationtuples.go:164-185)

    def _apply(self, ins: Sequence[RelationTuple], dels: Sequence[RelationTuple]) -> None:
        for t in list(ins) + list(dels):
            _check_subject(t)  # all-or-nothing: validated before anything changes
        if not ins and not dels:
            return
        for t in ins:  # writes, then deletes (relationtuples.go:260-270)
            sid = self._shard_id()
            self._rows.add((sid, t))
            self._by_tuple.setdefault(t, []).append(sid)
            self._p_ins[sid.int] = t
        for t in dels:
            self._remove_tuple(t)
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
            gone = {t for _, t in self._rows if query.matches(t)}
            for t in gone:
                self._remove_tuple(t)
            if gone:
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
        res: List[Tuple[uuid.UUID, RelationTuple]] = []
        with self._lock:
            for sid, t in self._rows.irange_key(min_key=last, inclusive=(False, True)):  # shard_id > lastID
                if query.matches(t):
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

    @staticmethod
    def _key(sid_int: int) -> int:
        return sid_int >> 64  # order key: the shard id's high 64 bits (uuid order up to a 2^-64 tie)

    def snapshot(self) -> Snapshot:
        """The snapshot of the current rows; refreshed on the first call after a write."""
        with self._lock:
            if self._snap is not None and self._snap_version == self._version:
                return self._snap
            delta = len(self._p_ins) + len(self._p_del)
            if self._snap is None or delta > max(4096, self.rebuild_fraction * len(self._rows)):
                arr = self.interner.tuples_array(t for _, t in self._rows)
                keys = np.fromiter((self._key(sid.int) for sid, _ in self._rows), np.uint64, len(self._rows))
                snap = Snapshot(arr, self.interner, self.program, self.device, devices=self.devices, keys=keys)
                self.rebuilds += 1
            else:
                ins = sorted(self._p_ins.items())
                ia = self.interner.tuples_array(t for _, t in ins)
                ik = np.fromiter((self._key(k) for k, _ in ins), np.uint64, len(ins))
                da = self.interner.tuples_array(self._p_del)
                snap = self._snap.apply(ia, da, ik)
                self.applies += 1
            self._snap, self._snap_version = snap, self._version
            self._p_ins, self._p_del = {}, set()
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
