"""Replicated snapshots (include/ketogpu.h device_mask / kg_snapshot_create_on): kg_check_batch and
kg_expand_batch split host-buffer batches over every replica inside the library -- one process
drives all of its GPUs, the way `keto serve` holds one check.Engine
(internal/driver/registry_default.go:180-185).  On a one-GPU box the replicas share device 0 (the
split, the per-replica lanes and the merge are the same code)."""
import threading

import numpy as np
import pytest

from keto_amd.engine import Config, Engine, ExpandEngine, Registry, Snapshot, queries_array
from oracle.oracle import POLICY_CANONICAL, Oracle
from test_gpu_check import random_graph, random_queries

pytestmark = pytest.mark.gpu


def _graph(seed=3, n_q=50_000):
    rng = np.random.default_rng(seed)
    it, tuples, nss, rels = random_graph(rng, n_obj=120, n_rows=1500)
    qs = random_queries(rng, nss, rels, 600, n_obj=120)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    idx = rng.integers(0, len(qs), n_q)
    depths = rng.integers(-1, 9, n_q)
    return it, tuples, q6[idx], depths


def test_replicas_split_matches_oracle():
    it, tuples, q6, depths = _graph()
    reg = Registry(tuples, [], interner=it, devices=[0, 0, 0])
    assert reg.snapshot.replicas() == [0, 0, 0]
    oracle = Oracle(it.tuples_array(tuples), it.wildcard_rel)
    for gmax in (2, 6):
        e = Engine(reg.snapshot, Config(gmax))
        out, err = e.batch_check_ids(queries_array(q6, depths), with_stats=True)
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL, nthreads=8)
        assert (out == exp).all() and (err == 0).all()
        assert e.last_stats["n_light"] + e.last_stats["n_no_holder"] > 0
        for n in (0, 1, 100, 16384 * 2 + 5):  # fewer queries than replicas x chunk, odd splits
            o2, _ = e.batch_check_ids(queries_array(q6[:n], depths[:n]))
            assert (o2 == exp[:n]).all(), n


def test_replicas_concurrent_callers():
    """Several host threads calling kg_check_batch on one replicated snapshot at once: every
    thread has its own lane (stream + pinned staging) per replica; answers are the serial ones."""
    it, tuples, q6, depths = _graph(seed=4, n_q=40_000)
    reg = Registry(tuples, [], interner=it, devices=[0, 0])
    e = Engine(reg.snapshot, Config(5))
    qa = queries_array(q6, depths)
    serial, _ = e.batch_check_ids(qa)
    fails, outs = [], {}

    def worker(k):
        try:
            for r in range(3):
                sl = slice(k * 5000, k * 5000 + 20000 + r * 7)
                o, er = e.batch_check_ids(qa[sl])
                assert (er == 0).all()
                outs[(k, r)] = (sl, o)
        except Exception as x:  # noqa: BLE001
            fails.append(x)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not fails, fails
    for (k, r), (sl, o) in outs.items():
        assert (o == serial[sl]).all(), (k, r)


def test_replicas_synthetic_and_expand():
    import torch
    from keto_amd import _lib
    from keto_amd.synth import hot_group_roots
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    one = Snapshot.synthetic(200_000, seed=20250131)
    two = Snapshot.synthetic(200_000, seed=20250131, devices=[0, 0])
    n = 60_000
    dq = torch.empty((n, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(one.handle, 5, n, dq.data_ptr()), "kg_synth_queries")
    q = dq.cpu().numpy().view(np.uint32)
    a, _ = Engine(one, Config(10)).batch_check_ids(q)
    b, _ = Engine(two, Config(10)).batch_check_ids(q)
    assert (a == b).all()
    roots = hot_group_roots(one.synth_ids(), 3000)
    ta = ExpandEngine(one, Config(4)).build_trees_ids(roots)
    tb = ExpandEngine(two, Config(4)).build_trees_ids(roots)
    for x, y in zip(ta, tb):
        assert (x is None and y is None) or (x.shape == y.shape and (x == y).all())
