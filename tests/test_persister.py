"""CPU tests: the snapshot persister's Manager surface (a restatement of the reference's
``relationtuple.ManagerTest``, internal/relationtuple/manager_requirements.go) and the request
batcher's dispatch logic.  No GPU: the snapshot is only built when an engine runs, and the
batcher is driven by a recording test double in place of the engine."""
import threading
import uuid

import numpy as np
import pytest

from keto_amd import _lib
from keto_amd.batcher import BatcherClosed, CheckBatcher
from keto_amd.ketoapi import RelationTuple, SubjectSet
from keto_amd.persister import (DEFAULT_PAGE_SIZE, MalformedPageToken, NilSubject, RelationQuery,
                                SnapshotPersister)


def ids(n, seed):
    r = np.random.default_rng(seed)
    return [str(uuid.UUID(int=int(r.integers(1 << 62)) << 64 | int(r.integers(1 << 62)))) for _ in range(n)]


def test_get_queries():
    # manager_requirements.go:57-169
    m = SnapshotPersister()
    u = ids(10, 1)
    tuples = [RelationTuple("ns", u[i % 2], f"r {i % 4}", subject_id=u[i]) for i in range(10)]
    m.write_relation_tuples(*tuples)
    cases = [
        (RelationQuery("ns"), tuples),
        (RelationQuery("ns", object=u[0]), tuples[0::2]),
        (RelationQuery("ns", relation="r 0"), [tuples[0], tuples[4], tuples[8]]),
        (RelationQuery("ns", object=u[0], relation="r 0"), [tuples[0], tuples[4], tuples[8]]),
        (RelationQuery("ns", subject_id=u[0]), [tuples[0]]),
        (RelationQuery("ns", object=u[0], subject_id=u[0]), [tuples[0]]),
        (RelationQuery("ns", relation="r 0", subject_id=u[0]), [tuples[0]]),
        (RelationQuery("ns", object=u[0], relation="r 0", subject_id=u[0]), [tuples[0]]),
    ]
    for q, want in cases:
        res, tok = m.get_relation_tuples(q)
        assert tok == ""
        assert sorted(map(str, res)) == sorted(map(str, want)), q


def test_pagination():
    # manager_requirements.go:171-227: page size 1 walks all 20 rows, token empty only on the last
    m = SnapshotPersister(seed=7)
    o = ids(1, 2)[0]
    tuples = [RelationTuple("ns", o, "r", subject_id=s) for s in ids(20, 3)]
    m.write_relation_tuples(*tuples)
    q = RelationQuery("ns", o, "r")
    seen, tok = [], ""
    for i in range(20):
        res, tok = m.get_relation_tuples(q, page_token=tok, page_size=1)
        assert len(res) == 1
        assert (tok == "") == (i == 19)
        seen += res
    assert sorted(map(str, seen)) == sorted(map(str, tuples))
    # pages of 7 cover the same rows in the same (shard) order
    pages, tok = [], ""
    while True:
        res, tok = m.get_relation_tuples(q, page_token=tok, page_size=7)
        pages += res
        if not tok:
            break
    assert pages == seen
    uuid.UUID(m.get_relation_tuples(q, page_size=1)[1])  # the token is a shard-id UUID (persister.go:123-125)


def test_default_page_size_and_empty_list():
    m = SnapshotPersister()
    m.write_relation_tuples(*[RelationTuple("ns", "o", "r", subject_id=f"u{i}") for i in range(DEFAULT_PAGE_SIZE + 1)])
    res, tok = m.get_relation_tuples(RelationQuery("ns"))
    assert len(res) == DEFAULT_PAGE_SIZE and tok
    res, tok = m.get_relation_tuples(RelationQuery("ns"), page_token=tok)
    assert len(res) == 1 and tok == ""
    assert m.get_relation_tuples(RelationQuery("other")) == ([], "")  # :229-240
    with pytest.raises(MalformedPageToken):
        m.get_relation_tuples(RelationQuery("ns"), page_token="not-a-uuid")


def test_delete():
    # manager_requirements.go:243-351
    m = SnapshotPersister()
    for rt in [RelationTuple("ns", "o", "r to delete", subject_id="s"),
               RelationTuple("ns", "o", "r to delete", subject_set=SubjectSet("ns", "x", "r2"))]:
        m.write_relation_tuples(rt)
        assert m.get_relation_tuples(RelationQuery("ns"))[0] == [rt]
        m.delete_relation_tuples(rt)
        assert m.get_relation_tuples(RelationQuery("ns"))[0] == []
    rs = [RelationTuple("ns", f"o{i}", f"r{i}", subject_id=f"s{i}") for i in range(4)]
    m.write_relation_tuples(*rs)
    m.delete_relation_tuples(rs[0], rs[2])
    assert sorted(map(str, m.get_relation_tuples(RelationQuery("ns"))[0])) == sorted(map(str, [rs[1], rs[3]]))
    rt = RelationTuple("n0", "o", "r", subject_set=SubjectSet("n1", "o", "r"))
    m.write_relation_tuples(rt)
    assert m.get_relation_tuples(RelationQuery("n0"))[0] == [rt]
    m.delete_relation_tuples(rt)
    assert m.get_relation_tuples(RelationQuery("n0"))[0] == []


def test_subject_kind_filter_and_duplicates():
    # whereSubject (relationtuples.go:124-145); no uniqueness constraint: duplicates are kept and
    # one delete removes all of them
    m = SnapshotPersister()
    a = RelationTuple("ns", "o", "r", subject_id="x")
    b = RelationTuple("ns", "o", "r", subject_set=SubjectSet("ns", "x", "r"))
    m.write_relation_tuples(a, a, b)
    assert len(m.get_relation_tuples(RelationQuery("ns"))[0]) == 3
    assert m.get_relation_tuples(RelationQuery(subject_id="x"))[0] == [a, a]
    assert m.get_relation_tuples(RelationQuery(subject_set=SubjectSet("ns", "x", "r")))[0] == [b]
    m.delete_relation_tuples(a)
    assert m.get_relation_tuples(RelationQuery("ns"))[0] == [b]
    m.write_relation_tuples(a)
    m.delete_all_relation_tuples(RelationQuery("ns", relation="r"))
    assert len(m) == 0


def test_transact():
    # manager_requirements.go:353-450
    m = SnapshotPersister()
    rs = [RelationTuple("ns", f"o{i}", f"r{i}", subject_id=f"s{i}") for i in range(4)]
    m.write_relation_tuples(rs[0], rs[1])
    m.transact_relation_tuples([rs[2], rs[3]], [rs[0]])
    assert sorted(map(str, m.get_relation_tuples(RelationQuery("ns"))[0])) == sorted(map(str, rs[1:]))
    m2 = SnapshotPersister()
    m2.write_relation_tuples(rs[0])
    v = m2.version
    bad = RelationTuple("ns", "o0", "r0")
    with pytest.raises(NilSubject):
        m2.transact_relation_tuples([bad], [rs[0]])
    with pytest.raises(NilSubject):
        m2.transact_relation_tuples([rs[1]], [bad])
    assert m2.get_relation_tuples(RelationQuery("ns"))[0] == [rs[0]] and m2.version == v  # rolled back


class RecordingEngine:
    """Test double for Engine.batch_check_ids: answers member iff obj id is even, error code
    7 when the relation id is 99; records every batch."""

    def __init__(self, delay=0.0):
        self.batches = []
        self.delay = delay
        self.lock = threading.Lock()

    def batch_check_ids(self, q):
        import time
        with self.lock:
            self.batches.append(q.copy())
        time.sleep(self.delay)
        out = np.where(q[:, 1] % 2 == 0, _lib.KG_IS_MEMBER, _lib.KG_NOT_MEMBER).astype(np.uint8)
        err = np.zeros(len(q), np.uint32)
        out[q[:, 2] == 99] = _lib.KG_ERROR
        err[q[:, 2] == 99] = 7
        return out, err


def test_batcher_many_threads():
    e = RecordingEngine(delay=0.002)
    n_threads, per = 8, 200
    got = {}
    with CheckBatcher(e, max_batch=128, max_wait_us=500) as b:
        def worker(k):
            fs = [(i, b.submit_ids([0, k * per + i, 1, 0xFFFFFFFF, 5, 0, 3])) for i in range(per)]
            for i, f in fs:
                got[k * per + i] = f.result(10)
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(n_threads)]
        [t.start() for t in ts]
        [t.join() for t in ts]
    assert len(got) == n_threads * per
    for obj, (res, err) in got.items():
        assert res == (_lib.KG_IS_MEMBER if obj % 2 == 0 else _lib.KG_NOT_MEMBER) and err == 0
    assert sum(len(x) for x in e.batches) == n_threads * per
    assert max(len(x) for x in e.batches) <= 128
    assert len(e.batches) < n_threads * per  # requests were actually coalesced
    assert b.latency_percentile(99) > 0


def test_batcher_errors_and_close():
    e = RecordingEngine()
    b = CheckBatcher(e, max_batch=4, max_wait_us=0)
    assert b.submit_ids([0, 2, 99, 0xFFFFFFFF, 1, 0, 0]).result(5) == (_lib.KG_ERROR, 7)
    fs = [b.submit_ids([0, i, 1, 0xFFFFFFFF, 1, 0, 0]) for i in range(10)]
    b.close()  # pending queries are still answered
    assert [f.result(5)[0] for f in fs] == [_lib.KG_IS_MEMBER if i % 2 == 0 else _lib.KG_NOT_MEMBER for i in range(10)]
    with pytest.raises(BatcherClosed):
        b.submit_ids([0, 0, 1, 0xFFFFFFFF, 1, 0, 0])

    class Broken:
        def batch_check_ids(self, q):
            raise _lib.KetoGPUError("boom")
    with CheckBatcher(Broken(), max_wait_us=0) as b2:
        with pytest.raises(_lib.KetoGPUError):
            b2.submit_ids([0, 0, 1, 0xFFFFFFFF, 1, 0, 0]).result(5)


def test_batcher_cancelled_future_keeps_dispatcher_alive():
    """A caller that cancels its future (e.g. a cancelled RPC) must not end the dispatcher."""
    e = RecordingEngine(delay=0.05)
    with CheckBatcher(e, max_batch=4, max_wait_us=20000) as b:
        f0 = b.submit_ids([0, 2, 1, 0xFFFFFFFF, 1, 0, 0])
        assert f0.cancel()  # still pending: cancellable
        f1 = b.submit_ids([0, 4, 1, 0xFFFFFFFF, 1, 0, 0])
        assert f1.result(5) == (_lib.KG_IS_MEMBER, 0)
        later = [b.submit_ids([0, i, 1, 0xFFFFFFFF, 1, 0, 0]) for i in range(6)]
        assert [f.result(5)[0] for f in later] == [_lib.KG_IS_MEMBER if i % 2 == 0 else _lib.KG_NOT_MEMBER
                                                    for i in range(6)]
    assert b.cancelled >= 1
    assert all(len(x) >= 1 for x in e.batches) and sum(len(x) for x in e.batches) == 7  # f0 never ran


def test_batcher_stats_are_bounded():
    e = RecordingEngine()
    with CheckBatcher(e, max_batch=1, max_wait_us=0) as b:
        b.STATS_WINDOW  # class constant
        for i in range(20):
            b.submit_ids([0, i, 1, 0xFFFFFFFF, 1, 0, 0]).result(5)
    assert b.batch_latency_s.maxlen == CheckBatcher.STATS_WINDOW and len(b.batch_latency_s) == 20


def test_interner_concurrent_fresh_strings_get_unique_ids():
    """Many threads interning fresh strings at once (the batcher's submit path): ids stay unique and
    resolve back to their own string."""
    from keto_amd.mapper import Interner
    it = Interner()
    n_threads, per = 8, 2000
    ids = [None] * n_threads
    start = threading.Barrier(n_threads)

    def worker(k):
        start.wait()
        # half the strings are shared between threads, half are private
        ids[k] = [(s, it.obj_id(s)) for s in
                  (f"shared{i}" if i % 2 else f"t{k}-{i}" for i in range(per))]
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(n_threads)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    by_str = {}
    for lst in ids:
        for s, v in lst:
            assert by_str.setdefault(s, v) == v  # one id per string
            assert it.obj_name(v) == s
    assert len(set(by_str.values())) == len(by_str)  # one string per id
    assert len(by_str) == n_threads * per // 2 + per // 2
