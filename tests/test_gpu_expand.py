"""GPU parity tests for batched expand (BuildTree): HIP path vs the reference's golden trees and the
CPU oracle.  Trees are compared exactly (same pre-order, same child order) against the oracle --
stronger than the reference's order-insensitive AssertInternalTreesAreEqual."""
import numpy as np
import pytest

from golden_cases import Case, all_cases
from keto_amd.engine import ExpandEngine, Registry, records_to_tree
from keto_amd.ketoapi import RelationTuple, SubjectSet, trees_equal_unordered
from keto_amd.mapper import SUBJECT_ID
from oracle.oracle import Oracle, records_to_tree as oracle_tree

pytestmark = pytest.mark.gpu

EXPAND_CASES = all_cases("expands")


@pytest.mark.parametrize("fn,case", EXPAND_CASES, ids=[f"{f}:{c['name']}" for f, c in EXPAND_CASES])
def test_golden_expand(fn, case):
    c = Case(case)
    reg = Registry(c.tuples, c.namespaces, interner=c.it)
    ex = reg.expand_engine()
    for e in case["expands"]:
        ex.config.max_read_depth = e["global_max_depth"]
        if e.get("subject_id") is not None:
            subject = e["subject_id"]
        else:
            ss = e["subject_set"]
            subject = SubjectSet(ss["namespace"], ss["object"], ss["relation"])
        got = ex.build_tree(subject, e["max_depth"])
        exp = Case.expected_tree(e)
        if e.get("ordered"):
            assert got == exp
        else:
            assert trees_equal_unordered(got, exp), (got, exp)


def _records(rec):
    return None if rec is None else np.asarray(rec, np.int64)


# (expand_gw, expand_skip_lds): default (16-lane walkers, then the 64-lane pass, gather-walk, hash pass);
# gather-walk on every root; hash pass on every root; the 64-lane pass on every root
GW_MODES = [(1, 0), (1, 1), (0, 1), (1, 2)]


@pytest.mark.parametrize("gw,skip", GW_MODES, ids=["default", "gw-all", "hash-all", "lds64-all"])
@pytest.mark.parametrize("seed", range(5))
def test_random_expand_vs_oracle(seed, gw, skip):
    rng = np.random.default_rng(50 + seed)
    n_obj = 30 + 30 * seed
    tuples = []
    for _ in range(200 + 300 * seed):
        ns, obj, rel = rng.choice(["a", "b"]), f"o{rng.integers(n_obj)}", rng.choice(["r0", "r1", "r2"])
        if rng.random() < 0.55:
            srel = rng.choice(["r0", "r1", "r2", "..."])
            s = f"({rng.choice(['a', 'b'])}:o{rng.integers(n_obj)}#{srel})"
        else:
            s = f"u{rng.integers(30)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    reg = Registry(tuples, [])
    reg.snapshot.tune("expand_gw", gw)
    reg.snapshot.tune("expand_skip_lds", skip)
    it = reg.interner
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    roots = []
    for _ in range(400):
        if rng.random() < 0.05:
            roots.append([SUBJECT_ID, it.obj_id(f"u{rng.integers(30)}"), 0, 0])
        else:
            roots.append([it.ns_id(rng.choice(["a", "b"])), it.obj_id(f"o{rng.integers(n_obj + 2)}"),
                          it.rel_id(rng.choice(["r0", "r1", "r2"])), int(rng.integers(-1, 7))])
    for gmax in (1, 2, 4, 7):
        ex = ExpandEngine(reg.snapshot)
        ex.config.max_read_depth = gmax
        arr = np.asarray(roots, np.int64)
        arr[:, 3] = arr[:, 3].astype(np.int32).view(np.uint32)
        got = ex.build_trees_ids(arr.astype(np.uint32))
        for r, g in zip(roots, got):
            exp = oracle.expand(r[0], r[1], r[2], r[3], gmax)
            _cmp_records(exp, g, (r, gmax))


@pytest.mark.parametrize("gw", [1, 0])
def test_expand_overflow_tier_and_wide_rows(gw):
    # a root whose visited set exceeds the LDS tier (pass 2: gather-walk or the HBM hash) and rows wider
    # than a wave
    tuples = [RelationTuple.from_string(f"g:root#m@(g:c{i}#m)") for i in range(900)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@(g:d{i % 300}#m)") for i in range(900)]
    tuples += [RelationTuple.from_string(f"g:d{i}#m@u{i}") for i in range(300)]
    tuples += [RelationTuple.from_string(f"g:c{i}#m@x{i}") for i in range(0, 900, 7)]
    reg = Registry(tuples, [])
    reg.snapshot.tune("expand_gw", gw)
    it = reg.interner
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    ex = reg.expand_engine()
    for gmax in (2, 3, 4):
        ex.config.max_read_depth = gmax
        got = ex.build_tree(SubjectSet("g", "root", "m"), 0)
        exp = oracle_tree(oracle.expand(it.ns_id("g"), it.obj_id("root"), it.rel_id("m"), 0, gmax), it)
        assert got == exp, gmax


def test_expand_gather_walk_large_slot_and_cycles():
    """A neighbourhood too large for a small gather-walk slot (96 k copied entries > 64 Ki): the root
    moves on to a large slot.  Shared grandchildren, back edges to the root and to a middle layer, and
    subject ids in every row make the visited order matter; depths 2..6 (the copy's reach D-2 and the
    local ids' reach D-1 both vary)."""
    tuples = [RelationTuple.from_string(f"g:root#m@(g:c{i}#m)") for i in range(320)]
    for i in range(320):
        for j in range(300):
            tuples.append(RelationTuple.from_string(f"g:c{i}#m@(g:d{(i * 7 + j * 13) % 2000}#m)"))
        tuples.append(RelationTuple.from_string(f"g:c{i}#m@u{i}"))
    for k in range(2000):
        tuples.append(RelationTuple.from_string(f"g:d{k}#m@(g:e{k % 50}#m)"))
        tuples.append(RelationTuple.from_string(f"g:d{k}#m@v{k}"))
        if k % 97 == 0:
            tuples.append(RelationTuple.from_string(f"g:d{k}#m@(g:root#m)"))
            tuples.append(RelationTuple.from_string(f"g:d{k}#m@(g:c{k % 320}#m)"))
    for k in range(50):
        tuples.append(RelationTuple.from_string(f"g:e{k}#m@(g:c{k}#m)"))
        tuples.append(RelationTuple.from_string(f"g:e{k}#m@w{k}"))
    reg = Registry(tuples, [])
    it = reg.interner
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    # (expand_gw, expand_gw_wait_us): default; large slots that never wait (their tickets are
    # abandoned and the roots go to the hash pass); no gather-walk
    for gw, wait in ((1, 100000), (1, 0), (0, 100000)):
        reg.snapshot.tune("expand_gw", gw)
        reg.snapshot.tune("expand_gw_wait_us", wait)
        ex = reg.expand_engine()
        for gmax in (2, 3, 4, 6):
            ex.config.max_read_depth = gmax
            got = ex.build_tree(SubjectSet("g", "root", "m"), 0)
            exp = oracle_tree(oracle.expand(it.ns_id("g"), it.obj_id("root"), it.rel_id("m"), 0, gmax), it)
            assert got == exp, (gw, wait, gmax)


def _cmp_records(exp, g, what):
    if exp is None:
        assert g is None, what
        return
    assert g is not None, what
    e2 = np.asarray(exp, np.int64).copy()
    g2 = np.asarray(g, np.int64).copy()
    ids = e2[:, 1] == 0  # SubjectIDs: oracle ns=rel=-1, GPU KG_SUBJECT_ID / 0
    e2[ids, 2] = 0
    e2[ids, 4] = 0
    g2[g2[:, 1] == 0, 2] = 0
    g2[g2[:, 1] == 0, 4] = 0
    assert e2.shape == g2.shape and (e2 == g2).all(), what


@pytest.mark.parametrize("n_tuples,gmax,gw,skip,wait", [(300_000, 5, 1, 0, 100000), (1_000_000, 3, 1, 0, 100000),
                                                         (300_000, 5, 1, 1, 100000), (300_000, 5, 0, 0, 100000),
                                                         (300_000, 5, 1, 0, 0), (300_000, 5, 1, 0, 50),
                                                         (300_000, 5, 1, 2, 100000)])
def test_c5_hot_group_roots_vs_oracle(n_tuples, gmax, gw, skip, wait):
    """Config C5's workload at reduced size: the generator's most popular group#member roots (the
    roots bench.py --mode expand times), expanded at the global depth, against the oracle's
    BuildTree on the snapshot's own rows -- same pre-order, same child order, every root."""
    from keto_amd.engine import Snapshot
    from keto_amd.synth import hot_group_roots
    snap = Snapshot.synthetic(n_tuples, seed=20250131)
    snap.tune("expand_gw", gw)
    snap.tune("expand_skip_lds", skip)
    snap.tune("expand_gw_wait_us", wait)  # 0 / 50 us: large slots give their tickets up
    roots = hot_group_roots(snap.synth_ids(), 1500)
    ex = ExpandEngine(snap)
    ex.config.max_read_depth = gmax
    got = ex.build_trees_ids(roots)
    oracle = Oracle(snap.export(), 0)
    big = 0
    for r, g in zip(roots, got):
        exp = oracle.expand(int(r[0]), int(r[1]), int(r[2]), 0, gmax)
        _cmp_records(exp, g, (r.tolist(), gmax))
        big += g is not None and len(g) > 512
    assert big > 0  # some trees outgrow the LDS pass (the hash / bitmap passes are exercised)


def test_expand_lane_memory_stays_flat():
    """A long-lived caller's lane keeps its device buffers, grown only when a call's output does not
    fit: 16 calls of the same batch on one thread allocate nothing after the first (the compacted-
    output buffer used to double on every call until hipMalloc failed, seen at C5 scale)."""
    import torch
    from keto_amd.engine import Snapshot
    from keto_amd.synth import hot_group_roots
    snap = Snapshot.synthetic(300_000, seed=20250131)
    roots = hot_group_roots(snap.synth_ids(), 2000)
    ex = ExpandEngine(snap)
    ex.config.max_read_depth = 5
    first = ex.build_trees_ids(roots)
    ex.build_trees_ids(roots)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    for _ in range(14):
        again = ex.build_trees_ids(roots)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info(0)[0]
    assert free0 - free1 < (64 << 20), (free0, free1)
    assert all((a is None and b is None) or (a == b).all() for a, b in zip(first, again))


@pytest.mark.parametrize("gw,skip", [(1, 0), (0, 1)], ids=["default", "hash-all"])
def test_expand_device_io_vs_oracle(gw, skip):
    """kg_expand_batch_device (roots and trees in HBM, offsets by a device scan): the same trees as the
    host-buffer call and the oracle's BuildTree, on C5 roots (giant trees included) and on random roots
    with nil trees and subject-id roots; an empty batch; the device output pool reused across calls."""
    import torch
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    from keto_amd.synth import hot_group_roots
    snap = Snapshot.synthetic(300_000, seed=20250131)
    snap.tune("expand_gw", gw)
    snap.tune("expand_skip_lds", skip)
    roots = hot_group_roots(snap.synth_ids(), 1500)
    rng = np.random.default_rng(7)
    extra = roots[rng.choice(len(roots), 64)].copy()
    extra[:16, 1] = 0x7FFFFFF0  # unknown objects: nil trees
    extra[16:24, 0] = SUBJECT_ID  # subject-id roots: a leaf each
    roots = np.concatenate([roots, extra])
    ex = ExpandEngine(snap)
    ex.config.max_read_depth = 5
    host = ex.build_trees_ids(roots)
    oracle = Oracle(snap.export(), 0)
    for k in range(2):  # the second call reuses the pool's buffers
        dev = ex.build_trees_ids(roots, device=True)
        for r, h, d in zip(roots, host, dev):
            assert (h is None) == (d is None) and (h is None or (h == d).all()), r.tolist()
    for r, d in zip(roots[:200], dev[:200]):
        if r[0] != SUBJECT_ID:
            _cmp_records(oracle.expand(int(r[0]), int(r[1]), int(r[2]), 0, 5), d, r.tolist())
    assert sum(d is not None and len(d) > 512 for d in dev) > 0
    # empty batch: root_off = [0]
    L = _lib.load()
    buf = _lib.kg_tree_buf()
    z = torch.zeros((1, 4), dtype=torch.int32, device="cuda:0")
    _lib.check(L.kg_expand_batch_device(snap.handle, z.data_ptr(), 0, 5, buf, None), "kg_expand_batch_device")
    off = np.ones(1, np.uint64)
    _lib.device_to_host(off, buf.root_off, 8)
    assert buf.n_nodes == 0 and off[0] == 0
    L.kg_tree_free(buf)
