"""GPU tests: the snapshot persister (writes invalidate the HBM snapshot; checks see every
committed write) and the request batcher (concurrent callers coalesced into kg_check_batch
calls), both against the CPU oracle on the persister's rows in shard order.  Bit-exact."""
import ctypes as C
import threading
import time

import numpy as np
import pytest

from keto_amd.batcher import CheckBatcher, NativeBatcher
from keto_amd.engine import queries_array
from keto_amd.ketoapi import RelationTuple, SubjectSet
from keto_amd.persister import RelationQuery, SnapshotPersister
from oracle.oracle import POLICY_CANONICAL, Oracle
from test_gpu_check import random_graph, random_queries

pytestmark = pytest.mark.gpu


def shard_rows(m: SnapshotPersister) -> np.ndarray:
    rows, tok = [], ""
    while True:
        page, tok = m.get_relation_tuples(RelationQuery(), page_token=tok, page_size=500)
        rows += page
        if not tok:
            return m.interner.tuples_array(rows)


@pytest.mark.parametrize("seed", range(3))
def test_persister_read_your_writes_vs_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    it, tuples, nss, rels = random_graph(rng, n_obj=50, n_rows=600)
    m = SnapshotPersister(interner=it, max_read_depth=6, seed=seed)
    e = m.permission_engine()
    qs = random_queries(rng, nss, rels, 1500, n_obj=50)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 8, len(qs))
    chunks = np.array_split(np.arange(len(tuples)), 3)
    for k, idx in enumerate(chunks):
        ins = [tuples[i] for i in idx]
        dels = [tuples[i] for i in rng.choice(chunks[k - 1], 40, replace=False)] if k else []
        m.transact_relation_tuples(ins, dels)
        out, err = e.batch_check_ids(queries_array(q6, depths))
        exp, oerr, _ = Oracle(shard_rows(m), it.wildcard_rel).check_batch(q6, depths, 6, POLICY_CANONICAL)
        assert (err == 0).all() and (oerr == 0).all()
        assert (out == exp).all(), np.nonzero(out != exp)[0][:10]
    assert m.rebuilds == 1 and m.applies == 2  # the first snapshot is built, then refreshed by deltas


def test_persister_write_delete_flip():
    m = SnapshotPersister()
    e = m.permission_engine()
    x = m.expand_engine()
    m.write_relation_tuples(RelationTuple.from_string("group:h#member@bob"))
    t = RelationTuple.from_string("doc:a#view@(group:g#member)")
    u = RelationTuple.from_string("group:g#member@alice")
    q = RelationTuple.from_string("doc:a#view@alice")
    m.write_relation_tuples(t)
    assert not e.check_is_member(q, 0)
    m.write_relation_tuples(u)
    assert e.check_is_member(q, 0)
    assert x.build_tree(SubjectSet("doc", "a", "view"), 0) is not None
    m.delete_relation_tuples(u)
    assert not e.check_is_member(q, 0)
    m.delete_all_relation_tuples(RelationQuery("doc"))
    assert x.build_tree(SubjectSet("doc", "a", "view"), 0) is None
    assert m.rebuilds + m.applies == 4 and m.applies >= 3
    assert e.check_is_member(RelationTuple.from_string("group:h#member@bob"), 0)


def test_batcher_vs_direct_batch():
    rng = np.random.default_rng(5)
    it, tuples, nss, rels = random_graph(rng, n_obj=80, n_rows=900)
    m = SnapshotPersister(interner=it, max_read_depth=5)
    m.write_relation_tuples(*tuples)
    e = m.permission_engine()
    qs = random_queries(rng, nss, rels, 4000, n_obj=80)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 7, len(qs))
    q7 = queries_array(q6, depths)
    want, _ = e.batch_check_ids(q7)
    exp, _, _ = Oracle(shard_rows(m), it.wildcard_rel).check_batch(q6, depths, 5, POLICY_CANONICAL)
    assert (want == exp).all()  # the direct batch is itself pinned to the oracle
    got = np.full(len(qs), 255, np.uint8)
    with CheckBatcher(e, max_batch=512, max_wait_us=300) as b:
        def worker(k):
            fs = [(i, b.submit_ids(q7[i])) for i in range(k, len(qs), 8)]
            for i, f in fs:
                got[i] = f.result(60)[0]
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        assert b.check_is_member(qs[0], int(depths[0])) == bool(want[0] == 1)
    assert (got == want).all()
    assert len(b.batch_sizes) < len(qs) and max(b.batch_sizes) <= 512


def test_persister_empty_snapshot():
    # every row deleted: the snapshot has no nodes; checks answer NotMember, expand a nil tree
    m = SnapshotPersister()
    t = RelationTuple.from_string("doc:a#view@alice")
    m.write_relation_tuples(t)
    e = m.permission_engine()
    assert e.check_is_member(t, 0)
    m.delete_relation_tuples(t)
    assert not e.check_is_member(t, 0)
    assert m.expand_engine().build_tree(SubjectSet("doc", "a", "view"), 0) is None


def test_native_batcher_many_callers_vs_oracle():
    """The library's request batcher (kg_batcher_check): 16 threads, each one blocking call per
    request (single checks and small bursts), against the oracle; rewrite errors come back per
    query; close answers what is pending and then refuses."""
    from keto_amd import _lib
    from keto_amd.engine import Registry
    from keto_amd.namespace import Namespace, Relation
    rng = np.random.default_rng(9)
    it, tuples, nss, rels = random_graph(rng, n_obj=80, n_rows=900)
    # namespace n0 declares r0, r1 only: queries reaching n0:*#r2 answer "relation not found"
    namespaces = [Namespace("n0", [Relation("r0"), Relation("r1")])]
    reg = Registry(tuples, namespaces, max_read_depth=5, interner=it, devices=[0, 0])
    qs = random_queries(rng, nss, rels, 3000, n_obj=80)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 7, len(qs))
    q7 = queries_array(q6, depths)
    exp, oerr, _ = Oracle(it.tuples_array(tuples), it.wildcard_rel, reg.program).check_batch(
        q6, depths, 5, POLICY_CANONICAL)
    assert (oerr != 0).any()
    got = np.full(len(qs), 255, np.uint8)
    gerr = np.zeros(len(qs), np.uint32)
    with NativeBatcher(reg.snapshot, 5, max_batch=256, max_wait_us=500, dispatchers=2) as nb:
        def worker(k):
            i = k
            while i < len(qs):
                n = 1 if k % 2 else min(5, len(qs) - i)  # odd threads: single checks, even: bursts
                sl = [i + j * 16 for j in range(n) if i + j * 16 < len(qs)]
                o, er = nb.check_ids(q7[sl])
                got[sl], gerr[sl] = o, er
                i += 16 * len(sl)
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        st = nb.stats()
        assert st["checks"] == len(qs) and st["batches"] < len(qs) and st["call_p99_ms"] > 0
        assert nb.check_is_member(qs[0], int(depths[0])) == bool(exp[0] == 1) or exp[0] == 2
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert (gerr.astype(np.int64) == oerr).all()
    with pytest.raises(_lib.KetoGPUError):
        nb2 = NativeBatcher(reg.snapshot, 5)
        nb2.L.kg_batcher_destroy(nb2._h)  # closed under the Python object: the next call must fail cleanly
        nb2._h = C.c_void_p()
        nb2.check_ids(q7[:1])


def _batcher_graph(seed=19):
    from keto_amd.engine import Registry
    rng = np.random.default_rng(seed)
    it, tuples, nss, rels = random_graph(rng, n_obj=80, n_rows=900)
    reg = Registry(tuples, [], max_read_depth=5, interner=it)
    qs = random_queries(rng, nss, rels, 2000, n_obj=80)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 7, len(qs))
    exp, _, _ = Oracle(it.tuples_array(tuples), it.wildcard_rel).check_batch(q6, depths, 5, POLICY_CANONICAL)
    return reg, queries_array(q6, depths), exp


def test_native_batcher_destroy_with_blocked_callers():
    """kg_batcher_destroy while 16 callers are blocked in kg_batcher_check (a batch that would only
    close after 5 s): destroy answers the pending batch, waits until every woken caller has left the
    call, and only then frees the batcher (the callers used to touch it after the free)."""
    reg, q7, exp = _batcher_graph()
    nb = NativeBatcher(reg.snapshot, 5, max_batch=1 << 20, max_wait_us=5_000_000, dispatchers=2)
    got = np.full(16 * 4, 255, np.uint8)
    errs = []
    entered = threading.Barrier(17)

    def worker(k):
        entered.wait()
        try:
            sl = list(range(4 * k, 4 * k + 4))
            o, _ = nb.check_ids(q7[sl])
            got[sl] = o
        except Exception as x:  # noqa: BLE001
            errs.append(x)

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    [t.start() for t in ts]
    entered.wait()
    time.sleep(0.3)  # every caller is inside kg_batcher_check, waiting on the open batch
    t0 = time.perf_counter()
    nb.close()
    assert time.perf_counter() - t0 < 4.0  # the batch closed on destroy, not on its 5 s deadline
    for t in ts:
        t.join(timeout=10)
        assert not t.is_alive()
    assert not errs, errs
    assert (got == exp[:64]).all()


@pytest.mark.parametrize("callers", [1, 16, 64])
def test_native_batcher_single_checks_vs_oracle(callers):
    """The drop-in CheckIsMember path of INTEGRATION.md: every request is ONE blocking
    kg_batcher_check of one query (handler.go:248-275 -> engine.go:54-60), from 1 / 16 / 64 caller
    threads; every answer equals the oracle; call and batch latency percentiles are reported."""
    reg, q7, exp = _batcher_graph(23)
    got = np.full(len(q7), 255, np.uint8)
    with NativeBatcher(reg.snapshot, 5, max_batch=4096, max_wait_us=200, dispatchers=4) as nb:
        def worker(k):
            for i in range(k, len(q7), callers):
                got[i] = nb.check_ids(q7[i:i + 1])[0][0]
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(callers)]
        t0 = time.perf_counter()
        [t.start() for t in ts]
        [t.join() for t in ts]
        el = time.perf_counter() - t0
        st = nb.stats()
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert st["checks"] == len(q7)
    if callers > 1:
        assert st["batches"] < len(q7)  # concurrent callers share batches
    print(f"batcher callers={callers}: {len(q7) / el:.0f} checks/s, call p50 {st['call_p50_ms']:.3f} ms "
          f"p99 {st['call_p99_ms']:.3f} ms, batch p99 {st['batch_p99_ms']:.3f} ms, "
          f"mean batch {st['checks'] / max(1, st['batches']):.1f}")


@pytest.mark.parametrize("seed,unions", [(0, False), (1, False), (2, True), (3, True)])
def test_incremental_refresh_matches_full_build(seed, unions):
    """kg_snapshot_apply after every transaction (inserts incl. new objects and subject sets,
    deletes of base rows and of rows inserted since the last snapshot, delete-all): checks equal
    the oracle on the persister's rows in shard order, and both checks and expand trees equal a
    snapshot built from scratch (kg_snapshot_create_ordered) from the same rows -- same shard order,
    so the same pre-order.  unions: a namespace program whose union rewrites are materialised."""
    from keto_amd.engine import Engine, ExpandEngine, Snapshot
    from keto_amd.mapper import SUBJECT_ID
    from test_gpu_check import random_program
    rng = np.random.default_rng(300 + seed)
    it, tuples, nss, rels = random_graph(rng, n_obj=60, n_rows=700)
    namespaces = random_program(rng, nss, rels, unions_only=True) if unions else []
    m = SnapshotPersister(namespaces=namespaces, interner=it, max_read_depth=5, seed=seed)
    base, rest = tuples[:400], tuples[400:]
    m.write_relation_tuples(*base)
    e = m.permission_engine()
    qs = random_queries(rng, nss, rels, 1200, n_obj=64)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 7, len(qs))
    roots = np.asarray([[it.ns_id(rng.choice(nss)), it.obj_id(f"o{rng.integers(64)}"), it.rel_id(rng.choice(rels)), 0]
                        for _ in range(150)], np.uint32)
    live = list(base)
    for step in range(6):
        ins = [rest.pop() for _ in range(min(len(rest), int(rng.integers(20, 60))))]
        ins += [RelationTuple.from_string(f"{rng.choice(nss)}:new{step}_{k}#{rng.choice(rels)}@u{k}") for k in range(3)]
        ins.append(RelationTuple.from_string(f"{nss[0]}:o{step}#{rels[0]}@({nss[1]}:new{step}_0#{rels[1]})"))
        dels = [live[i] for i in rng.choice(len(live), 15, replace=False)] if live else []
        m.transact_relation_tuples(ins, dels)
        live = [t for t in live + ins if t not in set(dels)]
        if step == 2:  # a row inserted since the last snapshot, deleted before the next one
            m.delete_relation_tuples(ins[0])
            live = [t for t in live if t != ins[0]]
        if step == 4:
            m.delete_all_relation_tuples(RelationQuery(namespace=nss[2]))
            live = [t for t in live if t.namespace != nss[2]]
        out, err = e.batch_check_ids(queries_array(q6, depths))
        rows = shard_rows(m)
        keys = np.fromiter((m._key(sid.int) for sid, _ in m._rows), np.uint64, len(m._rows))
        full = Snapshot(rows, it, m.program, keys=keys)
        fout, ferr = Engine(full, m.config).batch_check_ids(queries_array(q6, depths))
        assert (out == fout).all() and (err == ferr).all(), step
        exp, oerr, _ = Oracle(rows, it.wildcard_rel, m.program).check_batch(q6, depths, 5, POLICY_CANONICAL)
        assert (out == exp).all() and (err.astype(np.int64) == oerr).all(), (step, np.nonzero(out != exp)[0][:8])
        ga = ExpandEngine(m.snapshot(), m.config).build_trees_ids(roots)
        gb = ExpandEngine(full, m.config).build_trees_ids(roots)
        for a, b in zip(ga, gb):
            assert (a is None and b is None) or (a is not None and b is not None and np.array_equal(a, b)), step
    assert m.applies >= 5
