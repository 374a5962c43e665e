"""GPU parity tests for batched checks: the HIP path through the C ABI against the CPU oracle
and the reference's golden vectors.  Bit-exact (integer decisions)."""
import numpy as np
import pytest

from golden_cases import Case, all_cases
from keto_amd.engine import Config, Engine, Registry, Snapshot, queries_array
from keto_amd.ketoapi import RelationTuple
from keto_amd.mapper import Interner, SUBJECT_ID
from oracle.oracle import POLICY_CANONICAL, POLICY_DFS, Oracle

pytestmark = pytest.mark.gpu

CHECK_CASES = all_cases("checks")


@pytest.mark.parametrize("fn,case", CHECK_CASES, ids=[f"{f}:{c['name']}" for f, c in CHECK_CASES])
def test_golden_checks(fn, case):
    c = Case(case)
    reg = Registry(c.tuples, c.namespaces, interner=c.it)
    e = reg.permission_engine()
    for chk in case["checks"]:
        e.config.max_read_depth = chk["global_max_depth"]
        got = e.check_is_member(RelationTuple.from_string(chk["tuple"]), chk["max_depth"])
        assert got == chk["allowed"], chk


def random_graph(rng, n_obj=60, n_rows=400, n_ns=3, n_rel=3, p_set=0.45, p_wild=0.1, n_users=40):
    it = Interner()
    nss = [f"n{i}" for i in range(n_ns)]
    rels = [f"r{i}" for i in range(n_rel)]
    tuples = []
    for _ in range(n_rows):
        ns, obj, rel = rng.choice(nss), f"o{rng.integers(n_obj)}", rng.choice(rels)
        if rng.random() < p_set:
            srel = "..." if rng.random() < p_wild else rng.choice(rels)
            s = f"{rng.choice(nss)}:o{rng.integers(n_obj)}#{srel}"
        else:
            s = f"u{rng.integers(n_users)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    return it, tuples, nss, rels


def random_queries(rng, nss, rels, n, n_obj=60, n_users=40, p_setq=0.15):
    qs = []
    for _ in range(n):
        if rng.random() < p_setq:
            s = f"({rng.choice(nss)}:o{rng.integers(n_obj)}#{rng.choice(rels)})"
        else:
            s = f"u{rng.integers(n_users + 5)}"  # a few unknown subjects
        qs.append(RelationTuple.from_string(f"{rng.choice(nss)}:o{rng.integers(n_obj + 3)}#{rng.choice(rels)}@{s}"))
    return qs


@pytest.mark.parametrize("seed", range(20))
def test_random_graphs_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    it, tuples, nss, rels = random_graph(rng, n_obj=40 + 20 * (seed % 6), n_rows=200 + 150 * (seed % 6))
    reg = Registry(tuples, [], interner=it)
    # tier knobs (results never depend on them): a tiny per-query edge budget (queries overflow into
    # the backward / grid tiers mid-search), one / four / eight XCD steal ranges, and a backward tier
    # that hands nearly every query on (a one-edge reverse budget: the grid tier answers them)
    reg.snapshot.tune("stream_ecap", 6 if seed % 5 == 2 else 0)
    reg.snapshot.tune("stream_steal", 1 if seed % 3 == 1 else (8 if seed % 3 == 2 else 4))
    reg.snapshot.tune("back_edges", 1 if seed % 4 == 3 else 0)
    qs = random_queries(rng, nss, rels, 3000, n_obj=40 + 20 * (seed % 6))
    depths = rng.integers(-1, 9, len(qs))
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    for gmax in (1, 3, 5, 8):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths))
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        assert (err == 0).all() and (oerr == 0).all()
        bad = np.nonzero(out != exp)[0]
        assert bad.size == 0, [(str(qs[i]), int(depths[i]), int(out[i]), int(exp[i])) for i in bad[:10]]
        # schedule sensitivity: queries where the Go DFS schedule agrees are bit-exact with it too
        dfs, _, _ = oracle.check_batch(q6, depths, gmax, POLICY_DFS)
        inv = dfs == exp
        assert (out[inv] == dfs[inv]).all()


@pytest.mark.parametrize("ecap", [512, 0, 3])
def test_stream_tier_long_rows_and_dense_cycles(ecap):
    """Rows longer than a FIFO entry holds (2047 edges), dense cycles (the direct-mapped visited cache
    evicts and re-expands), many queries per wave on one hub: exact vs the oracle."""
    rng = np.random.default_rng(77)
    tuples = [RelationTuple.from_string(f"g:hub#m@(g:c{i}#m)") for i in range(2500)]  # > 2047-edge row
    tuples += [RelationTuple.from_string(f"g:c{i}#m@(g:c{(i * 7 + 3) % 2500}#m)") for i in range(2500)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@(g:k{i % 40}#m)") for i in range(0, 2500, 3)]
    tuples += [RelationTuple.from_string(f"g:k{i}#m@(g:k{(i + 1) % 40}#m)") for i in range(40)]  # a 40-cycle
    tuples += [RelationTuple.from_string(f"g:k{i}#m@u{i}") for i in range(0, 40, 5)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@v{i % 97}") for i in range(0, 2500, 11)]
    reg = Registry(tuples, [])
    reg.snapshot.tune("stream_ecap", ecap)
    it = reg.interner
    qs = [RelationTuple.from_string(f"g:{r}#m@{u}") for r in ["hub", "k0", "k3", "c5", "c17", "c999"]
          for u in ["u0", "u35", "v3", "v96", "nobody"]]
    q6 = np.asarray([it.tuple_ids(t) for t in qs] * 40, np.uint32)
    depths = rng.integers(0, 12, len(q6))
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    for gmax in (3, 6, 12):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
        exp, _, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        assert (out == exp).all() and (err == 0).all(), (gmax, np.nonzero(out != exp)[0][:10])


def test_heavy_path_overflow_star():
    # one query reaching > LDS capacity (512 visited) leaves the wave tiers (backward / grid tier)
    tuples = [RelationTuple.from_string(f"g:root#m@(g:c{i}#m)") for i in range(3000)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@(g:d{i % 700}#m)") for i in range(3000)]
    tuples += [RelationTuple.from_string("g:d699#m@target"), RelationTuple.from_string("g:c5#m@near")]
    reg = Registry(tuples, [])
    e = reg.permission_engine()
    it = reg.interner
    qs = [RelationTuple.from_string(s) for s in
          ["g:root#m@target", "g:root#m@near", "g:root#m@nobody", "g:c1#m@target", "g:d699#m@target"]]
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    for gmax in (2, 3, 4, 6):
        e.config.max_read_depth = gmax
        out, _ = e.batch_check_ids(queries_array(q6, 0), with_stats=True)
        exp, _, _ = oracle.check_batch(q6, np.zeros(len(qs), np.int32), gmax)
        assert list(out) == list(exp), (gmax, out, exp)
    assert e.last_stats["n_heavy"] + e.last_stats["n_back"] >= 1


@pytest.mark.parametrize("back_edges,grid_cap", [(1, 0), (0, 0), (1, 600), (1, 5000)])
def test_tail_tiers_backward_and_grid(back_edges, grid_cap):
    # > 512 enqueued edges leaves the stream tier; the backward tier (reverse search from the
    # subject's holders) answers first and hands on what outgrows it to the grid tier -- with a
    # one-edge reverse budget (back_edges 1) nearly everything goes on to the grid tier
    tuples = [RelationTuple.from_string(f"g:root#m@(g:c{i}#m)") for i in range(5000)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@(g:d{i % 1500}#m)") for i in range(5000)]
    tuples += [RelationTuple.from_string(f"g:d{i}#m@(g:e{i % 400}#m)") for i in range(1500)]
    tuples += [RelationTuple.from_string("g:e399#m@target"), RelationTuple.from_string("g:d7#m@mid")]
    # a second root with ~1000 expanded nodes: beyond the wave tier, inside the LDS workgroup tier
    tuples += [RelationTuple.from_string(f"g:r2#m@(g:f{i}#m)") for i in range(1000)]
    tuples += [RelationTuple.from_string(f"g:f{i}#m@(g:h{i % 100}#m)") for i in range(1000)]
    tuples += [RelationTuple.from_string("g:h99#m@deep")]
    # a subject held by ~1900 nodes whose parents outgrow the backward tier's LDS (-> forward)
    tuples += [RelationTuple.from_string(f"g:d{i}#m@pop") for i in range(1500)]
    tuples += [RelationTuple.from_string(f"g:e{i}#m@pop") for i in range(400)]
    reg = Registry(tuples, [])
    e = reg.permission_engine()
    e.snapshot.tune("back_edges", back_edges)
    # grid_cap: the workspace's grid log holds 600 / 5000 entries, so rounds overflow, rerun with
    # fewer slots, and the queries that overflow it alone run in the shared full-size pool (the
    # per-query rounds: MS-BFS off); grid_cap 0 runs the grid tier's queries as MS-BFS (kg_msbfs.hip)
    e.snapshot.tune("grid_cap", grid_cap)
    e.snapshot.tune("grid_ms", 0 if grid_cap else 1)
    it = reg.interner
    qs = [RelationTuple.from_string(s) for s in
          ["g:root#m@target", "g:root#m@mid", "g:root#m@none", "g:c3#m@target", "g:c7#m@mid", "g:d3#m@target",
           "g:r2#m@deep", "g:r2#m@none", "g:root#m@pop", "g:r2#m@pop", "g:root#m@deep"]]
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    tiers = {"n_heavy": 0, "n_back": 0, "n_no_holder": 0}
    for gmax in (2, 3, 4, 5, 6):
        e.config.max_read_depth = gmax
        out, _ = e.batch_check_ids(queries_array(q6, 0), with_stats=True)
        exp, _, _ = oracle.check_batch(q6, np.zeros(len(qs), np.int32), gmax)
        assert list(out) == list(exp), (gmax, out, exp)
        for k in tiers:
            tiers[k] += e.last_stats[k]
    assert tiers["n_heavy"] >= 1, tiers
    assert tiers["n_no_holder"] >= 1 and (back_edges == 1 or tiers["n_back"] >= 1), tiers


def test_empty_and_unknown():
    reg = Registry([RelationTuple.from_string("a:b#c@d")], [])
    e = reg.permission_engine()
    out, err = e.batch_check_ids(np.zeros((0, 7), np.uint32))
    assert out.shape == (0,)
    assert e.check_is_member(RelationTuple.from_string("a:b#c@d"), 0)
    assert not e.check_is_member(RelationTuple.from_string("a:b#c@zzz"), 0)
    assert not e.check_is_member(RelationTuple.from_string("x:y#z@d"), 0)  # unknown namespace -> false


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.parametrize("n_tuples,gmax,ecap", [(200_000, 10, 512), (300_000, 5, 512), (300_000, 10, 32),
                                                 (300_000, 5, 0), (300_000, 5, 32)])
def test_synthetic_graph_vs_oracle(n_tuples, gmax, ecap):
    """ecap: the stream tier's per-query edge budget (32: most long walks go on to the backward and
    grid tiers; 0: no budget, every walk finishes in the stream tier)."""
    torch = _torch()
    from keto_amd import _lib
    snap = Snapshot.synthetic(n_tuples, seed=20250131)
    snap.tune("stream_ecap", ecap)
    n = 20000
    dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 7, n, dq.data_ptr()), "kg_synth_queries")
    e = Engine(snap, Config(gmax))
    q = dq.cpu().numpy().view(np.uint32)
    out, err = e.batch_check_ids(q, with_stats=True)
    assert (err == 0).all()
    rows = snap.export()
    oracle = Oracle(rows, 0)
    exp, _, _ = oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
    assert (out == exp).all(), np.nonzero(out != exp)[0][:10]
    frac = out.mean()
    assert 0.05 < frac < 0.95  # both answers occur
    # layered generator => every query is schedule-invariant
    dfs, _, _ = oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_DFS, nthreads=8)
    assert (dfs == exp).all()


@pytest.mark.parametrize("ecap", [512, 32])
def test_adjx_layouts_vs_oracle(ecap, monkeypatch):
    """The snapshot's adjx in node order (KG_ADJX_ORDER=0: parallel to adj) and hot-first (the default,
    round 5: rows in descending in-degree order, begins from DevSnap::adjx_off): the same answers, equal
    to the oracle's -- through the stream tier and, at ecap 32, the backward and grid tiers that follow
    adjx records and node-map row begins too."""
    torch = _torch()
    from keto_amd import _lib
    n, gmax = 20000, 10
    outs = []
    for order in ("0", "1"):
        monkeypatch.setenv("KG_ADJX_ORDER", order)  # read when the snapshot builds its hash tables
        snap = Snapshot.synthetic(300_000, seed=20250131)
        snap.tune("stream_ecap", ecap)
        dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
        _lib.check(_lib.load().kg_synth_queries(snap.handle, 11, n, dq.data_ptr()), "kg_synth_queries")
        q = dq.cpu().numpy().view(np.uint32)
        out, err = Engine(snap, Config(gmax)).batch_check_ids(q)
        assert (err == 0).all()
        outs.append(out)
        if order == "1":
            exp, _, _ = Oracle(snap.export(), 0).check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL,
                                                              nthreads=8)
            assert (out == exp).all(), np.nonzero(out != exp)[0][:10]
        snap.close()
    assert (outs[0] == outs[1]).all()
    assert 0.05 < outs[1].mean() < 0.95


@pytest.mark.parametrize("stream_wgs,grid_wgs", [(1, 1), (3, 8)])
def test_occupancy_knobs_vs_oracle(stream_wgs, grid_wgs):
    """k_stream4 / k_grid_level workgroups per CU (defaults 2 / 2): fewer or more waves draining the
    stream tier's per-XCD work lists and spreading a grid level, the same answers."""
    torch = _torch()
    from keto_amd import _lib
    snap = Snapshot.synthetic(300_000, seed=20250131)
    snap.tune("stream_wgs", stream_wgs)
    snap.tune("grid_wgs", grid_wgs)
    snap.tune("stream_ecap", 64)
    snap.tune("grid_ms", 0)  # the per-query grid rounds (the MS-BFS tier takes >= 4 workgroups per CU)
    n = 20000
    dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 23, n, dq.data_ptr()), "kg_synth_queries")
    q = dq.cpu().numpy().view(np.uint32)
    e = Engine(snap, Config(10))
    out, err = e.batch_check_ids(q, with_stats=True)
    assert (err == 0).all()
    exp, _, _ = Oracle(snap.export(), 0).check_batch(q[:, :6], q[:, 6].view(np.int32), 10, POLICY_CANONICAL,
                                                     nthreads=8)
    assert (out == exp).all(), np.nonzero(out != exp)[0][:10]


@pytest.mark.parametrize("back_edges,back_wgs", [(32, 3), (4096, 1), (1 << 16, 2)])
def test_backward_budget_vs_oracle(back_edges, back_wgs):
    """The backward tier's reverse-edge budget (kg_snapshot_tune back_edges; default 2^12) and its
    workgroup count: a tiny budget hands most backward walks on to the grid tier, a large one keeps
    hub-heavy ones in the wave; one workgroup per CU makes waves take a second query.  Answers equal
    the oracle's whatever tier finishes a query."""
    torch = _torch()
    from keto_amd import _lib
    snap = Snapshot.synthetic(300_000, seed=20250131)
    snap.tune("stream_ecap", 32)  # most long walks leave the stream tier
    snap.tune("back_edges", back_edges)
    snap.tune("back_wgs", back_wgs)
    n = 20000
    dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 11, n, dq.data_ptr()), "kg_synth_queries")
    q = dq.cpu().numpy().view(np.uint32)
    e = Engine(snap, Config(10))
    out, err = e.batch_check_ids(q, with_stats=True)
    assert (err == 0).all()
    exp, _, _ = Oracle(snap.export(), 0).check_batch(q[:, :6], q[:, 6].view(np.int32), 10, POLICY_CANONICAL,
                                                     nthreads=8)
    assert (out == exp).all(), np.nonzero(out != exp)[0][:10]
    st = e.last_stats
    assert st["n_back"] > 0 and st["n_heavy"] + st["n_back"] > 0, st


@pytest.mark.parametrize("n,mat", [(2049, 0), (2304, 1), (4352, 0), (6100, 1), (2305, 0)])
def test_small_batches_mixed_routes_vs_oracle(n, mat, monkeypatch):
    """Batches just past a multiple of 2048 queries: the stream tier's work list has 8 shards of
    ceil(blocks / 8) * 256 records, more than 8 n u32 when n is small (the round-3 scratch layout gave
    the list only 8 n u32, so shard 7 overwrote the general and hand-on lists).  The batch
    mixes rewrite queries (general route, the interpreter's list), stream-tier queries and, with a
    tiny edge budget, many hand-ons to the backward / grid tiers."""
    from keto_amd.namespace import compile_program
    monkeypatch.setenv("KG_MATERIALIZE", str(mat))  # 0: unions through the interpreter too (more general queries)
    rng = np.random.default_rng(n)
    it, tuples, nss, rels = random_graph(rng, n_obj=300, n_rows=3000, n_users=60)
    namespaces = random_program(rng, nss, rels)  # every rewrite kind: interpreter, formula split, unions
    prog = compile_program(namespaces, it, lower_ttu=False)  # the oracle: TTU leaves as written
    reg = Registry(tuples, namespaces, interner=it)
    reg.snapshot.tune("stream_ecap", 1)  # a root row of >= 2 set edges hands the query on at once
    qs = random_queries(rng, nss, rels, n, n_obj=300, n_users=60)
    depths = rng.integers(-1, 9, len(qs))
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, prog)
    e = Engine(reg.snapshot, Config(6))
    out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
    st = e.last_stats
    exp, oerr, _ = oracle.check_batch(q6, depths, 6, POLICY_CANONICAL)
    bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
    assert bad.size == 0, (bad.size, [(str(qs[i]), int(depths[i]), int(out[i]), int(exp[i]), int(err[i]), int(oerr[i]))
                                      for i in bad[:10]])
    # the routes the batch mixes (after the parity check, so a mismatch is reported first)
    assert st["n_light"] > 0 and st["n_heavy"] + st["n_back"] > 0, st
    if not mat:
        assert st["n_general"] > 0, st


def test_concurrent_streams_match_serial():
    """kg_check_batch_device on several streams at once (one workspace per stream, one host thread
    per stream, the way bench.py keeps batches in flight) gives exactly the serial answers."""
    import threading
    torch = _torch()
    from keto_amd import _lib
    import ctypes as C
    L = _lib.load()
    snap = Snapshot.synthetic(300_000, seed=20250131)
    n, P, gmax = 30000, 3, 10
    streams = [torch.cuda.Stream() for _ in range(P)]
    dqs = []
    for p in range(P):
        q = torch.empty((n, 7), dtype=torch.int32, device="cuda")
        _lib.check(L.kg_synth_queries(snap.handle, 100 + p, n, q.data_ptr()), "kg_synth_queries")
        dqs.append(q)
    e = Engine(snap, Config(gmax))
    serial = [e.batch_check_ids(q.cpu().numpy().view(np.uint32))[0] for q in dqs]
    outs = [[torch.full((n,), 7, dtype=torch.uint8, device="cuda") for _ in range(4)] for _ in range(P)]
    errs = [torch.full((n,), 99, dtype=torch.int32, device="cuda") for _ in range(P)]
    torch.cuda.synchronize()
    failures = []

    def worker(p):
        try:
            for r in range(4):
                _lib.check(L.kg_check_batch_device(snap.handle, dqs[p].data_ptr(), n, gmax, outs[p][r].data_ptr(),
                                                   errs[p].data_ptr(), None, C.c_void_p(streams[p].cuda_stream)),
                           "kg_check_batch_device")
            streams[p].synchronize()
        except Exception as x:  # noqa: BLE001
            failures.append(x)

    th = [threading.Thread(target=worker, args=(p,)) for p in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not failures, failures
    for p in range(P):
        assert (errs[p].cpu().numpy() == 0).all()
        for r in range(4):
            assert (outs[p][r].cpu().numpy() == serial[p]).all(), (p, r)
    q0 = dqs[0].cpu().numpy().view(np.uint32)
    exp, _, _ = Oracle(snap.export(), 0).check_batch(q0[:, :6], q0[:, 6].view(np.int32), gmax, POLICY_CANONICAL,
                                                      nthreads=8)
    assert (serial[0] == exp).all()


# ---------------------------------------------------------------- rewrites (interpreter path)
from keto_amd.namespace import (ComputedSubjectSet, InvertResult, Namespace, Relation,  # noqa: E402
                                SubjectSetRewrite, TupleToSubjectSet)


def random_program(rng, nss, rels, unions_only=False):
    """Random namespace configs: computed children only point to lower relation indexes (acyclic).
    unions_only: `or` of computed / tuple-to-subject-set children (nested), the shape rewrite
    materialisation (kg_augment.hip) turns into plain union nodes."""
    def child(level, own):
        if unions_only:
            k = rng.integers(3 if level < 2 else 2)
            if k == 0 and own > 0:
                return ComputedSubjectSet(rels[rng.integers(own)])
            if k < 2:
                return TupleToSubjectSet(rng.choice(rels), rng.choice(rels))
            return SubjectSetRewrite([child(level + 1, own) for _ in range(rng.integers(1, 3))], "or")
        k = rng.integers(4 if level < 2 else 3)
        if k == 0 and own > 0:
            return ComputedSubjectSet(rels[rng.integers(own)])
        if k == 1 or (k == 0 and own == 0):
            return TupleToSubjectSet(rng.choice(rels), rng.choice(rels))
        if k == 2:
            return InvertResult(child(level + 1, own))
        return SubjectSetRewrite([child(level + 1, own) for _ in range(rng.integers(1, 4))],
                                 "and" if rng.random() < 0.4 else "or")

    out = []
    for ns in nss:
        relations = []
        for j, r in enumerate(rels):
            rw = None
            if rng.random() < 0.5:
                rw = SubjectSetRewrite([child(0, j) for _ in range(rng.integers(1, 3))],
                                       "and" if rng.random() < 0.3 and not unions_only else "or")
            relations.append(Relation(r, rewrite=rw))
        out.append(Namespace(ns, relations))
    return out


@pytest.mark.parametrize("mat", [1, 0])
@pytest.mark.parametrize("unions", [False, True])
@pytest.mark.parametrize("seed", range(8))
def test_random_rewrites_vs_oracle(seed, unions, mat, monkeypatch):
    """Random programs (all rewrite kinds, or unions only) on random graphs with undeclared
    relations, with rewrite materialisation on (default) and off (KG_MATERIALIZE=0)."""
    from keto_amd.namespace import compile_program
    monkeypatch.setenv("KG_MATERIALIZE", str(mat))
    rng = np.random.default_rng(100 + seed + (1000 if unions else 0))
    nss = ["a", "b", "c"]
    rels = ["r0", "r1", "r2", "r3"]
    it = Interner()
    namespaces = random_program(rng, nss, rels, unions_only=unions)
    prog = compile_program(namespaces, it, lower_ttu=False)  # the oracle: TTU leaves as written
    n_obj, n_users = 30 + 10 * seed, 25
    tuples = []
    for _ in range(150 + 60 * seed):
        ns, obj = rng.choice(nss), f"o{rng.integers(n_obj)}"
        rel = rng.choice(rels) if rng.random() < 0.97 else "undeclared"
        if rng.random() < 0.5:
            srel = rng.choice(rels + ["..."]) if rng.random() < 0.98 else "undeclared"
            s = f"({rng.choice(nss)}:o{rng.integers(n_obj)}#{srel})"
        else:
            s = f"u{rng.integers(n_users)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    reg = Registry(tuples, namespaces, interner=it)
    qs = random_queries(rng, nss, rels, 2000, n_obj=n_obj, n_users=n_users)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(-1, 7, len(qs))
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, prog)
    for gmax in (1, 2, 4, 6):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
        assert bad.size == 0, [(str(qs[i]), int(depths[i]), int(out[i]), int(err[i]), int(exp[i]), int(oerr[i]))
                               for i in bad[:10]]
    m = reg.snapshot.materialized()
    if not mat:
        assert m["union_nodes"] == 0
    elif unions:
        assert m["union_nodes"] > 0, m


@pytest.mark.parametrize("preset", [0, 1])
def test_packed_device_vs_device(preset):
    """kg_check_batch_packed_device (round 5: 16-B queries in HBM): without a namespace program (C2's
    generator) k_resolve reads the packed rows itself; with one (C3's OPL program: formula split, union
    nodes) they are unpacked on the device first.  Answers and error codes equal kg_check_batch_device's
    on the same queries, and the oracle's."""
    torch = _torch()
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from keto_amd import _lib
    L = _lib.load()
    n, gmax = 20000, 10
    snap = Snapshot.synthetic(300_000 if preset == 0 else 150_000, seed=20250131, preset=preset)
    dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
    _lib.check(L.kg_synth_queries(snap.handle, 13, n, dq.data_ptr()), "kg_synth_queries")
    dp = bench.pack_queries_device(dq)
    dl = torch.empty_like(dp)  # the library's packer (kg_pack_queries_device) gives the same rows
    _lib.check(L.kg_pack_queries_device(snap.handle, dq.data_ptr(), n, dl.data_ptr(), None), "kg_pack_queries_device")
    assert torch.equal(dl.cpu(), dp.cpu())
    o1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    e1 = torch.empty(n, dtype=torch.int32, device="cuda")
    o2, e2 = torch.empty_like(o1), torch.empty_like(e1)
    _lib.check(L.kg_check_batch_device(snap.handle, dq.data_ptr(), n, gmax, o1.data_ptr(), e1.data_ptr(), None, None),
               "kg_check_batch_device")
    _lib.check(L.kg_check_batch_packed_device(snap.handle, dp.data_ptr(), n, gmax, o2.data_ptr(), e2.data_ptr(), None,
                                              None), "kg_check_batch_packed_device")
    torch.cuda.synchronize()
    a, b = o1.cpu().numpy(), o2.cpu().numpy()
    assert (a == b).all() and (e1.cpu().numpy() == e2.cpu().numpy()).all()
    q = dq.cpu().numpy().view(np.uint32)
    exp, oerr, _ = Oracle(snap.export(), 0, snap.program if preset else None).check_batch(
        q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
    assert (b == exp).all() and (oerr == 0).all()
    assert 0.05 < b.mean() < 0.95


@pytest.mark.parametrize("seed", [0, 5])
def test_packed_boundary_vs_oracle(seed):
    """kg_check_batch_packed (16-B packed queries in, answers as bytes, error codes as
    sparse (index, code) pairs of the KG_ERROR answers): the same answers and codes as kg_check_batch and
    the oracle, on random programs with undeclared relations (many errors) -- 20 k queries, so the error
    list outgrows its read-back prefetch (4096 pairs) and the queries span several staging slices; and
    a truncated list (err_cap 5) keeps the full count and the first pairs by index."""
    from keto_amd import _lib
    from keto_amd.namespace import compile_program
    rng = np.random.default_rng(700 + seed)
    nss, rels = ["a", "b", "c"], ["r0", "r1", "r2", "r3"]
    it = Interner()
    namespaces = random_program(rng, nss, rels)
    prog = compile_program(namespaces, it, lower_ttu=False)
    n_obj = 60
    tuples = []
    for _ in range(600):
        ns, obj = rng.choice(nss), f"o{rng.integers(n_obj)}"
        rel = rng.choice(rels) if rng.random() < 0.9 else "undeclared"
        s = f"({rng.choice(nss)}:o{rng.integers(n_obj)}#{rng.choice(rels + ['undeclared'])})" if rng.random() < 0.5 \
            else f"u{rng.integers(25)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    reg = Registry(tuples, namespaces, interner=it)
    qs = random_queries(rng, nss, rels + ["undeclared"], 2000, n_obj=n_obj, n_users=25)
    q6 = np.tile(np.asarray([it.tuple_ids(t) for t in qs], np.uint32), (10, 1))
    depths = np.tile(rng.integers(-1, 7, len(qs)), 10)
    q = queries_array(q6, depths)
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, prog)
    for gmax in (2, 5):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(q)
        pout, pairs, n_err = e.batch_check_packed(q)
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        assert (pout == out).all() and (out == exp).all() and (err.astype(np.int64) == oerr).all()
        bad = np.nonzero(out == _lib.KG_ERROR)[0]
        assert n_err == bad.size > 4096, (n_err, bad.size)
        assert (pairs[:, 0] == bad).all() and (pairs[:, 1] == err[bad]).all()
        t_out, t_pairs, t_n = e.batch_check_packed(q, err_cap=5)
        assert (t_out == out).all() and t_n == n_err and (t_pairs == pairs[:5]).all()


def test_relation_not_found_and_cycle():
    nss = [Namespace("d", [Relation("a"), Relation("b", rewrite=SubjectSetRewrite([ComputedSubjectSet("c")])),
                           Relation("c", rewrite=SubjectSetRewrite([ComputedSubjectSet("b")]))])]
    tuples = [RelationTuple.from_string(s) for s in ["d:x#a@u", "d:x#a@(d:y#zz)", "d:y#a@u"]]
    reg = Registry(tuples, nss)
    e = reg.permission_engine()
    assert e.check_is_member(RelationTuple.from_string("d:x#a@u"), 0)
    r = e.check_relation_tuple(RelationTuple.from_string("d:x#a@v"), 0)  # reaches undeclared d:y#zz
    assert r.err is not None and r.err.code == 1
    r = e.check_relation_tuple(RelationTuple.from_string("d:x#b@u"), 0)  # b -> c -> b
    assert r.err is not None and r.err.code == 3
    r = e.check_relation_tuple(RelationTuple.from_string("d:x#nope@u"), 0)
    assert r.err is not None and r.err.code == 1


@pytest.mark.parametrize("n_tuples,gmax,cap2,mat", [(150_000, 10, 0, 1), (250_000, 5, 0, 1), (150_000, 10, 32, 1),
                                                  (150_000, 10, 0, 0), (150_000, 10, 32, 0)])
def test_synthetic_c3_rewrites_vs_oracle(n_tuples, gmax, cap2, mat, monkeypatch):
    """Config C3: the Drive-like graph + folder forest + OPL view/edit/share.  Materialised
    (default): view / edit are union nodes answered by the rewrite-free tiers, share = view &
    !blocked goes through the interpreter, whose computed `view` is one BFS from the union node.
    mat = 0: every query through the interpreter.  cap2 = 32: the many-slot HBM pass holds 32
    nodes per BFS, so what reaches it overflows into the single full-size slot (pass 3)."""
    torch = _torch()
    from keto_amd import _lib
    monkeypatch.setenv("KG_MATERIALIZE", str(mat))
    snap = Snapshot.synthetic(n_tuples, seed=20250131, preset=1)
    m = snap.materialized()
    assert (m["union_nodes"] > 0) == bool(mat), m
    snap.tune("interp_cap2", cap2)
    n = 6000
    dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 11, n, dq.data_ptr()), "kg_synth_queries")
    e = Engine(snap, Config(gmax))
    q = dq.cpu().numpy().view(np.uint32)
    out, err = e.batch_check_ids(q, with_stats=True)
    if mat:  # view / edit are union nodes, share = view & !blocked splits into two leaf checks
        assert e.last_stats["n_general"] < n // 20, e.last_stats
    else:
        assert e.last_stats["n_general"] == n
    oracle = Oracle(snap.export(), 0, snap.program)
    exp, oerr, _ = oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
    bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
    assert bad.size == 0, [(q[i].tolist(), int(out[i]), int(exp[i]), int(err[i]), int(oerr[i])) for i in bad[:8]]
    assert 0.05 < (out == 1).mean() < 0.95 and (out == 2).sum() == 0
    dfs, _, _ = oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_DFS, nthreads=8)
    assert (dfs == exp).all()  # rewrites sit outside every visited scope: schedule-invariant


@pytest.mark.parametrize("mat", [1, 0])
@pytest.mark.parametrize("seed", range(4))
def test_formula_rewrites_vs_oracle(seed, mat, monkeypatch):
    """Boolean rewrites over union / plain relations (kg_formula.hip): and / or / not over computed
    leaves split into leaf checks run by the rewrite-free tiers; formulas with a tuple-to-subject-set
    leaf, a non-union rewrite leaf or an undeclared leaf, objects whose own node holds rows, and a
    union that reaches an undeclared relation stay with the interpreter.  Bit-exact with the oracle,
    materialisation on and off."""
    from keto_amd.namespace import compile_program
    monkeypatch.setenv("KG_MATERIALIZE", str(mat))
    rng = np.random.default_rng(500 + seed)
    C, T, N, O = ComputedSubjectSet, TupleToSubjectSet, InvertResult, SubjectSetRewrite
    rels = [Relation("a"), Relation("b"), Relation("blocked"), Relation("parent"),
            Relation("u1", rewrite=O([C("a"), T("parent", "u1")])),
            Relation("u2", rewrite=O([C("b"), C("u1")])),
            Relation("f1", rewrite=O([C("u1"), N(C("blocked"))], "and")),
            Relation("f2", rewrite=O([O([C("u2"), N(C("a"))], "and"), C("blocked")])),
            Relation("f3", rewrite=O([N(C("u1"))])),
            Relation("f4", rewrite=O([C("u1"), T("parent", "f1")], "and")),
            Relation("f5", rewrite=O([C("a"), C("f1")], "and")),
            Relation("f6", rewrite=O([C("u2"), C("und")], "and")),
            Relation("f7", rewrite=O([N(O([C("a"), C("b")], "and")), N(C("u2"))], "and")),
            Relation("u3", rewrite=O([C("a"), T("parent", "zz")]))]
    namespaces = [Namespace("d", rels)]
    it = Interner()
    prog = compile_program(namespaces, it, lower_ttu=False)  # the oracle: TTU leaves as written
    n_obj, n_users = 40 + 20 * seed, 20
    tuples = []
    for _ in range(400 + 150 * seed):
        x = f"d:o{rng.integers(n_obj)}"
        k = rng.integers(10)
        if k < 3:
            tuples.append(f"{x}#parent@(d:o{rng.integers(n_obj)}#...)")
        elif k < 8:
            r = ["a", "b", "blocked", "a", "b"][k - 3]
            subj = f"u{rng.integers(n_users)}" if rng.random() < 0.7 else f"(d:o{rng.integers(n_obj)}#u2)"
            tuples.append(f"{x}#{r}@{subj}")
        elif k == 8:
            tuples.append(f"{x}#f1@u{rng.integers(n_users)}")  # own rows: not split
        else:
            tuples.append(f"{x}#parent@(d:o{rng.integers(n_obj)}#...)")
    tuples = [RelationTuple.from_string(t) for t in tuples]
    reg = Registry(tuples, namespaces, interner=it)
    qrels = ["a", "u1", "u2", "u3", "f1", "f2", "f3", "f4", "f5", "f6", "f7"]
    qs = [RelationTuple.from_string(f"d:o{rng.integers(n_obj)}#{rng.choice(qrels)}@u{rng.integers(n_users + 2)}")
          for _ in range(3000)]
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(-1, 7, len(qs))
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, prog)
    general = []
    for gmax in (1, 2, 3, 5, 7):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
        assert bad.size == 0, [(str(qs[i]), int(depths[i]), int(out[i]), int(err[i]), int(exp[i]), int(oerr[i]))
                               for i in bad[:10]]
        general.append(e.last_stats["n_general"])
        assert 0.05 < (out == 1).mean() < 0.95
    if mat:  # f1 / f2 / f3 / f7 queries on objects without own rows split (and u1 / u2 are union nodes)
        assert max(general) < 0.75 * len(qs), general


@pytest.mark.parametrize("cap2", [0, 32, 700])
def test_rewrite_bfs_beyond_lds(cap2):
    # a computed-subject-set rewrite above a rewrite-free subtree of ~3,700 nodes: the
    # interpreter's BFS run outgrows the LDS pass (512 nodes) and reruns in the many-slot HBM hash
    # pass; cap2 = 32 / 700 make that pass overflow too, so the query finishes in pass 3
    nss = [Namespace("g", [Relation("m"), Relation("v", rewrite=SubjectSetRewrite([ComputedSubjectSet("m")]))])]
    tuples = [RelationTuple.from_string(f"g:root#m@(g:c{i}#m)") for i in range(3000)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@(g:d{i % 700}#m)") for i in range(3000)]
    tuples += [RelationTuple.from_string("g:d699#m@target"), RelationTuple.from_string("g:c5#m@near")]
    reg = Registry(tuples, nss)
    reg.snapshot.tune("interp_cap2", cap2)
    e = reg.permission_engine()
    it = reg.interner
    qs = [RelationTuple.from_string(s) for s in
          ["g:root#v@target", "g:root#v@near", "g:root#v@nobody", "g:c1#v@target", "g:root#m@target",
           "g:root#v@(g:d3#m)", "g:c9#v@nobody"]]
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, reg.program)
    for gmax in (2, 3, 4, 6):
        e.config.max_read_depth = gmax
        for rep in range(2):  # the second batch reuses slots whose tables the first one left
            out, err = e.batch_check_ids(queries_array(q6, 0), with_stats=True)
            exp, oerr, _ = oracle.check_batch(q6, np.zeros(len(qs), np.int32), gmax, POLICY_CANONICAL)
            assert list(out) == list(exp) and list(err) == list(oerr), (gmax, rep, out, exp)


def test_opl_full_example_rewrites_vs_oracle():
    """The reference parser's golden AST (internal/schema/.snapshots/TestParser-suite=snapshots-
    full_example.json, a tests/golden fixture) loaded through namespace_from_json, compiled, and
    evaluated by the GPU interpreter on a random graph over its namespaces: bit-exact with the
    oracle, error codes included (the "not" permission and nested and/or/traverse)."""
    import json
    import os
    from keto_amd.namespace import compile_program, namespace_from_json
    golden = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                         "opl_full_example.json")))
    namespaces = [namespace_from_json({"name": n, "relations": rels}) for n, rels in sorted(golden.items())]
    it = Interner()
    prog = compile_program(namespaces, it, lower_ttu=False)  # the oracle: TTU leaves as written
    rng = np.random.default_rng(2024)
    files, folders, groups, users = [f"f{i}" for i in range(60)], [f"d{i}" for i in range(20)], \
        [f"g{i}" for i in range(15)], [f"u{i}" for i in range(30)]
    tuples = []
    for _ in range(700):
        k = rng.integers(9)
        f = rng.choice(files)
        if k == 0:
            tuples.append(f"File:{f}#parents@(File:{rng.choice(files)}#...)")
        elif k == 1:
            tuples.append(f"File:{f}#parents@(Folder:{rng.choice(folders)}#...)")
        elif k == 2:
            tuples.append(f"File:{f}#viewers@{rng.choice(users)}")
        elif k == 3:
            tuples.append(f"File:{f}#viewers@(Group:{rng.choice(groups)}#members)")
        elif k == 4:
            tuples.append(f"File:{f}#owners@{rng.choice(users)}")
        elif k == 5:
            tuples.append(f"File:{f}#siblings@(File:{rng.choice(files)}#...)")
        elif k == 6:
            tuples.append(f"Folder:{rng.choice(folders)}#viewers@(Group:{rng.choice(groups)}#members)")
        elif k == 7:
            tuples.append(f"Group:{rng.choice(groups)}#members@{rng.choice(users)}")
        else:
            tuples.append(f"Group:{rng.choice(groups)}#members@(Group:{rng.choice(groups)}#members)")
    tuples = [RelationTuple.from_string(t) for t in tuples]
    reg = Registry(tuples, namespaces, interner=it)
    assert reg.snapshot.program is not None
    qs = []
    for _ in range(3000):
        rel = rng.choice(["view", "edit", "not", "rename", "viewers", "owners", "parents"])
        ns, obj = ("Folder", rng.choice(folders)) if rng.random() < 0.2 else ("File", rng.choice(files))
        subj = rng.choice(users + ["nobody"]) if rng.random() < 0.9 else f"(Group:{rng.choice(groups)}#members)"
        qs.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{subj}"))
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(-1, 8, len(qs))
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel, prog)
    for gmax in (2, 5, 8):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
        assert bad.size == 0, [(str(qs[i]), int(depths[i]), int(out[i]), int(exp[i]), int(err[i]), int(oerr[i]))
                               for i in bad[:8]]
        assert e.last_stats["n_general"] > 0
        assert 0 < (exp == 1).sum() and (exp == 0).sum() > 0


@pytest.mark.parametrize("preset,n_tuples", [(0, 2_000_000), (1, 600_000)])
def test_bench_tune_set_vs_oracle(preset, n_tuples):
    """The exact engine configuration bench.py times (bench.apply_tune with bench.py's default
    arguments: stream variant, edge budget, stream_steal, back_wgs, stream_wgs, grid_wgs, grid_reserve,
    device_sync), with the bench's batches in flight on their own streams through
    kg_check_batch_device: every answer of every batch equals the oracle (Go-order DFS and canonical)."""
    import ctypes as C
    import threading
    import bench
    torch = _torch()
    from keto_amd import _lib
    L = _lib.load()
    a = bench.parse(["--preset", str(preset)])
    snap = Snapshot.synthetic(n_tuples, seed=20250131, preset=preset)
    bench.apply_tune(snap, a)
    assert snap.tuned["back_wgs"] == (1 if preset else 3) and snap.tuned["stream_steal"] == 4
    P, n, gmax = a.inflight, 50_000, a.global_depth
    streams = [torch.cuda.Stream() for _ in range(P)]
    dqs = []
    for p in range(2 * P):
        q = torch.empty((n, 7), dtype=torch.int32, device="cuda")
        _lib.check(L.kg_synth_queries(snap.handle, 300 + p, n, q.data_ptr()), "kg_synth_queries")
        dqs.append(q)
    outs = [torch.full((n,), 7, dtype=torch.uint8, device="cuda") for _ in range(2 * P)]
    errs = [torch.full((n,), 99, dtype=torch.int32, device="cuda") for _ in range(2 * P)]
    torch.cuda.synchronize()
    failures = []

    def worker(p):
        try:
            for k in (p, p + P):
                st = _lib.kg_stats()
                _lib.check(L.kg_check_batch_device(snap.handle, dqs[k].data_ptr(), n, gmax, outs[k].data_ptr(),
                                                   errs[k].data_ptr(), C.byref(st) if k == p else None,
                                                   C.c_void_p(streams[p].cuda_stream)), "kg_check_batch_device")
            streams[p].synchronize()
        except Exception as x:  # noqa: BLE001
            failures.append(x)

    th = [threading.Thread(target=worker, args=(p,)) for p in range(P)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not failures, failures
    oracle = Oracle(snap.export(), 0, snap.program if preset else None)
    for k in range(2 * P):
        q = dqs[k].cpu().numpy().view(np.uint32)
        out, err = outs[k].cpu().numpy(), errs[k].cpu().numpy()
        exp, oerr, _ = oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
        bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
        assert bad.size == 0, (k, bad[:10])
        if k < 2:
            dfs, _, _ = oracle.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_DFS, nthreads=8)
            assert (dfs == exp).all()
        assert 0.05 < (out == 1).mean() < 0.95


@pytest.mark.parametrize("ms,grid_cap,seed,tg_cap", [
    (0, 0, 0, 256), (0, 0, 1, 256), (0, 700, 2, 256), (0, 60, 3, 256), (0, 0, 4, 256), (8, 0, 0, 256), (1, 0, 1, 256),
    (1, 40, 2, 256), (2, 300, 3, 256), (8, 0, 5, 256), (16, 0, 6, 256), (4, 120, 7, 256), (8, 0, 8, 0), (1, 0, 9, 3)])
def test_grid_dense_vs_oracle(ms, grid_cap, seed, tg_cap):
    """The grid tier on dense graphs with cycles, hubs and subjects held only by rows nothing points
    at: a tiny stream-tier edge budget and a one-edge backward budget send nearly every query there;
    every depth 2..9 is bit-exact with the oracle.  ms 0: the per-query rounds (kg_grid.hip), with a
    log small enough that rounds overflow and rerun (grid_cap); ms 1: the
    multi-source bit-parallel BFS (kg_msbfs.hip, 64 x ms queries per group), with
    level buffers small enough that rounds overflow and rerun with fewer groups, or that one group
    overflows them alone and the list falls back to the per-query rounds (grid_cap as grid_ms_cap);
    ms = 64-bit words per node mask (64 queries each: 1 word = ~40 groups of the batch's grid
    queries, 16 words = one group); tg_cap = holders above which a query's subject is probed in
    dset per newly reached node instead of marked in the target masks (0: every query probed)."""
    rng = np.random.default_rng(900 + seed)
    n_obj, n_users = 120, 60
    tuples = []
    for i in range(n_obj):
        for _ in range(int(rng.integers(1, 14))):  # dense set edges, cycles included
            tuples.append(f"g:o{i}#m@(g:o{int(rng.integers(n_obj))}#m)")
        if rng.random() < 0.3:
            tuples.append(f"g:o{i}#m@u{int(rng.integers(n_users))}")
    for i in range(40):  # docs: roots that nothing points at, holding users directly too
        for _ in range(int(rng.integers(1, 8))):
            tuples.append(f"d:x{i}#v@(g:o{int(rng.integers(n_obj))}#m)")
        tuples.append(f"d:x{i}#v@w{int(rng.integers(20))}")  # w*: held only by docs
    tuples = [RelationTuple.from_string(t) for t in tuples]
    reg = Registry(tuples, [])
    snap = reg.snapshot
    snap.tune("stream_ecap", 3)
    snap.tune("back_edges", 1)  # the backward tier hands nearly every query on to the grid tier
    snap.tune("grid_ms", 1 if ms else 0)
    if ms:
        snap.tune("grid_ms_words", ms)
        snap.tune("grid_ms_tg_cap", tg_cap)
    snap.tune("grid_ms_cap" if ms else "grid_cap", grid_cap)
    it = reg.interner
    qs = []
    for _ in range(2500):
        root = f"d:x{int(rng.integers(40))}#v" if rng.random() < 0.6 else f"g:o{int(rng.integers(n_obj))}#m"
        r = rng.random()
        subj = f"u{int(rng.integers(n_users))}" if r < 0.7 else (f"w{int(rng.integers(20))}" if r < 0.9
                                                                  else f"(g:o{int(rng.integers(n_obj))}#m)")
        qs.append(RelationTuple.from_string(f"{root}@{subj}"))
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 10, len(qs))
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    grid, allowed = 0, []
    for gmax in (2, 3, 4, 5, 6, 9):
        e = Engine(snap, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
        exp, _, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        bad = np.nonzero(out != exp)[0]
        assert bad.size == 0 and (err == 0).all(), (gmax, [(str(qs[i]), int(depths[i]), int(out[i]), int(exp[i]))
                                                            for i in bad[:8]])
        grid += e.last_stats["n_grid"]
        allowed.append(out.mean())
    assert grid > 1000
    assert 0.01 < min(allowed) and 0.2 < max(allowed) < 0.99, allowed
