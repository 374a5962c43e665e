"""Hash-sharded mode: keto_amd.sharded's level/exchange protocol.

CPU (gloo, world_size 2 and 3): ShardedChecker over the test-only restatement of the local steps
(tests/shard_ref.py) against the C oracle on the full graph -- exercises the all-gather of bucket
sizes, the all-to-all of records, hit reports to the home rank, termination and the bucket-overflow
rerun.  GPU: the HIP local steps (kg_shard_seed / kg_shard_level) at world_size 1 and 2 (two
processes on one GPU, gloo exchange) against the same oracle, bit-exact."""
import os
import time
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph(seed, n_obj=50, n_rows=500):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_check import random_graph, random_queries  # noqa: E402  (pure-python helpers)
    from keto_amd.engine import queries_array
    rng = np.random.default_rng(seed)
    it, tuples, nss, rels = random_graph(rng, n_obj=n_obj, n_rows=n_rows)
    qs = random_queries(rng, nss, rels, 400, n_obj=n_obj)
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(-1, 8, len(qs))
    return it, it.tuples_array(tuples), queries_array(q6, depths)


def _expected(t6, wildcard, q, gmax):
    from oracle.oracle import POLICY_CANONICAL, Oracle
    o = Oracle(t6, wildcard)
    exp, err, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
    assert (err == 0).all()
    return exp


def _cpu_worker(rank, world, port, seed, cap, outq, budget=0, back_budget=1 << 14, protocol="auto"):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from keto_amd.sharded import ShardedChecker
    from shard_ref import CpuShardOps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    it, t6, q = _graph(seed)
    ops = CpuShardOps(t6, it.wildcard_rel, rank, world, budget=budget, back_budget=back_budget)
    mine = np.array_split(np.arange(len(q)), world)[rank]  # this rank's slice of the batch
    chk = ShardedChecker(ops, rank, world, dist, device="cpu", cap=cap, protocol=protocol)
    out = {}
    for gmax in (2, 5):
        syncs = chk.host_syncs
        res, err = chk.check(torch.from_numpy(q[mine].view(np.int32).copy()), gmax)
        out[gmax] = (mine, res.numpy().copy(), chk.cap, chk.back_levels, chk.final_levels, chk.host_syncs - syncs,
                     chk.levels)
    outq.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cap,budget,back_budget,protocol",
                         [(2, 1 << 12, 0, 0, "dynamic"), (3, 4, 0, 0, "dynamic"), (2, 1 << 12, 0, 0, "fixed"),
                          (3, 4, 0, 0, "fixed"), (3, 1 << 12, 0, 0, "auto"), (2, 1 << 12, 2, 1 << 14, "auto"),
                          (3, 8, 1, 1 << 14, "auto"), (2, 1 << 12, 1, 2, "auto")])
def test_sharded_protocol_gloo(world, cap, budget, back_budget, protocol):
    """cap=4 / 8 force bucket overflows: every rank must rerun the batch with larger buckets.  budget
    1 / 2: nearly every expanding query escalates, so the backward phase (all-gathered reverse hops
    from the subject's holders) decides it; back_budget 2: most of those go on to the final forward
    phase.  protocol "fixed" (the default without escalation): fixed-size buckets, gdepth + 1 levels,
    no host round trip inside a batch (at most 2 per batch: the first batch of a size reads the
    done-bitmap width, and the end-of-batch readback; a rerun after an overflow adds one)."""
    seed = 3
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cpu_worker, args=(r, world, port, seed, cap, outq, budget, back_budget, protocol))
          for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    it, t6, q = _graph(seed)
    for gmax in (2, 5):
        exp = _expected(t6, it.wildcard_rel, q, gmax)
        res = np.zeros(len(q), np.uint8)
        for _, out in got:
            mine, r, final_cap, back_levels, final_levels, syncs, levels = out[gmax]
            res[mine] = r
            if cap <= 8:
                assert final_cap > cap
            if protocol == "fixed" or (protocol == "auto" and not budget):
                assert levels == gmax + 1
                if cap > 8:
                    assert syncs <= 2, syncs
            if budget and gmax == 5:
                assert back_levels > 0
            if back_budget == 2 and gmax == 5:
                assert final_levels > 0
        assert (res == exp).all(), np.nonzero(res != exp)[0][:10]
        assert 0 < exp.mean() < 1


ASYM_SIZES = [(10, 250), (10, 5), (300, 5), (0, 200), (150, 0), (150, 37), (37, 37)]  # per call: (rank 0, rank 1)


def _cpu_asym_worker(rank, world, port, seed, outq, protocol):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from keto_amd.sharded import ShardedChecker
    from shard_ref import CpuShardOps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    it, t6, q = _graph(seed)
    chk = ShardedChecker(CpuShardOps(t6, it.wildcard_rel, rank, world), rank, world, dist, device="cpu", cap=1 << 12,
                         protocol=protocol)
    out = []
    for sizes in ASYM_SIZES:
        lo = sum(sizes[:rank])
        mine = np.arange(lo, lo + sizes[rank])
        res, err = chk.check(torch.from_numpy(q[mine].view(np.int32).copy().reshape(-1, 7)), 4)
        out.append((mine, res.numpy().copy(), err.numpy().copy()))
    outq.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("protocol", ["fixed", "dynamic"])
def test_sharded_asymmetric_batches_gloo(protocol):
    """Per-rank batch sizes that differ and change asymmetrically from call to call (a rank with no
    query at all included): every rank must issue the same collectives in the same order on every
    batch (a per-rank cache of the slot count let one rank skip an all-reduce another rank
    issued), and the answers equal the oracle's."""
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cpu_asym_worker, args=(r, 2, port, 4, outq, protocol)) for r in range(2)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=240) for _ in range(2)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    it, t6, q = _graph(4)
    exp = _expected(t6, it.wildcard_rel, q, 4)
    for _, out in got:
        for mine, r, e in out:
            assert (e == 0).all() and (r == exp[mine]).all(), mine[:5]


def test_owner_matches_library():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from keto_amd import _lib
    from shard_ref import shard_owner
    L = _lib.load()
    for ns, obj, n in [(0, 0, 8), (1, 12345, 8), (3, 2 ** 31 - 2, 7), (2, 99, 1), (65534, 5, 64)]:
        assert L.kg_shard_owner(ns, obj, n) == shard_owner(ns, obj, n)


class _LibAdapter:
    """keto_amd.sharded.LibShardedChecker (the whole batch inside libketogpu.so) with ShardedChecker's
    counters, so the same workers and assertions run both drivers."""

    def __init__(self, snap, rank, world, dist_, transport):
        from keto_amd.sharded import LibShardedChecker
        self.chk = LibShardedChecker(snap, rank, world, dist_, transport=transport)
        self.levels = self.host_syncs = self.back_levels = self.general_queries = 0
        self.path = None
        self.reruns = {1: 0, 2: 0}

    def check(self, dq, gmax):
        r = self.chk.check(dq, gmax)
        st = self.chk.stats()
        self.levels = st["levels"]
        self.back_levels = st["escalation_levels"]
        self.path = st["path"]
        self.host_syncs += st["host_syncs"]
        self.reruns[1] += st["reruns_bucket"]
        self.reruns[2] += st["reruns_visited"]
        self.general_queries += st["general_queries"]
        return r


# (host round trips, levels) of a clean in-library batch by path: local-first tier chain, one-rank device
# level loop, exchange protocol (at most gdepth + 1 exchanges -- a batch after the first runs the count
# learned from the one before, its last non-empty exchange + 2; the agreement all-reduce and the
# end-of-batch one)
LIB_PATH_COST = {0: lambda g: (0, 0), 1: lambda g: (1, g), 2: lambda g: (2, g + 1)}


def _checker(driver, snap, rank, world, dist_, cap=256):
    """driver "py": keto_amd.sharded.ShardedChecker over the kg_shard_* steps; "lib[-rccl|-host][-loop]
    [-forced]": the in-library batch over RCCL (default at world 1) or the gloo host transport (default at
    world > 1: ranks share the one GPU, which RCCL does not allow).  World 1 runs local-first (the replica
    tier chain) unless "-loop" (kg_snapshot_tune shard_local 0: the one-rank device level loop) or
    "-forced" (shard_force_exchange 1: the N > 1 exchange protocol over the transport, each rank its own
    peer)."""
    from keto_amd.sharded import HipShardOps, ShardedChecker
    if driver == "py":
        return ShardedChecker(HipShardOps(snap), rank, world, dist_, device="cuda", cap=cap)
    parts = driver.split("-")
    transport = "rccl" if "rccl" in parts else ("host" if "host" in parts else ("rccl" if world == 1 else "host"))
    if "loop" in parts:
        snap.tune("shard_local", 0)
    if "forced" in parts:
        snap.tune("shard_force_exchange", 1)
    return _LibAdapter(snap, rank, world, dist_, transport)


# ------------------------------------------------------------------ GPU (HIP local steps)
def _gpu_worker(rank, world, port, seed, outq, budget=None, back_budget=None):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import HipShardOps, ShardedChecker
    dist_ = None
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)  # two ranks on one GPU: host-staged
        dist_ = dist
    torch.cuda.set_device(0)
    it, t6, q = _graph(seed, n_obj=80, n_rows=1500)
    snap = Snapshot(t6, it, None, 0, shard=(rank, world))
    if budget is not None:
        snap.tune("shard_budget", budget)
    if back_budget is not None:
        snap.tune("shard_back_budget", back_budget)
    mine = np.array_split(np.arange(len(q)), world)[rank]
    chk = ShardedChecker(HipShardOps(snap), rank, world, dist_, device="cuda", cap=256)
    out = {}
    for gmax in (1, 3, 6):
        dq = torch.from_numpy(q[mine].view(np.int32).copy()).cuda()
        res, err = chk.check(dq, gmax)
        out[gmax] = (mine, res.cpu().numpy(), err.cpu().numpy())
    outq.put((rank, out))
    if dist_:
        dist.destroy_process_group()


def _run_gpu(world, seed, budget=None, back_budget=None):
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gpu_worker, args=(r, world, port, seed, outq, budget, back_budget))
          for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=100) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    it, t6, q = _graph(seed, n_obj=80, n_rows=1500)
    for gmax in (1, 3, 6):
        exp = _expected(t6, it.wildcard_rel, q, gmax)
        res = np.zeros(len(q), np.uint8)
        for _, out in got:
            mine, r, e = out[gmax]
            assert (e == 0).all()
            res[mine] = r
        assert (res == exp).all(), (gmax, np.nonzero(res != exp)[0][:10])


@pytest.mark.gpu
@pytest.mark.parametrize("world,budget,back_budget", [(1, None, None), (2, None, None), (1, 1, None), (2, 2, None),
                                                     (1, 0, None), (1, 1, 2), (2, 1, 2)])
def test_sharded_hip_vs_oracle(world, budget, back_budget):
    """Random graphs (cycles, subject sets as subjects), against the oracle.  Budgets 1 / 2 escalate
    nearly every query that expands to the backward phase (reverse search from the subject's holders
    over all-gathered records); 0 turns escalation off; back_budget 2 sends most of them on to the
    final forward phase."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_gpu(world, seed=11, budget=budget, back_budget=back_budget)


# ------------------------------------------------------------------ rewrites reached in sharded mode
def _impure_graph(seed):
    """A random graph plus a namespace program: relation r2 of n1 has a rewrite and r1 of n2 is
    declared while r2 is not (undeclared) -> relflag != 0 for (n1, r2), (n2, r0), (n2, r2)."""
    sys.path.insert(0, ROOT)
    from keto_amd.namespace import ComputedSubjectSet, Namespace, Relation, SubjectSetRewrite, compile_program
    it, t6, q = _graph(seed, n_obj=40, n_rows=400)
    nss = [Namespace("n1", [Relation("r0"), Relation("r1"),
                            Relation("r2", rewrite=SubjectSetRewrite([ComputedSubjectSet("r0")]))]),
           Namespace("n2", [Relation("r1")])]
    prog = compile_program(nss, it)
    impure = [(it.ns_id("n1"), it.rel_id("r2")), (it.ns_id("n2"), it.rel_id("r0")), (it.ns_id("n2"), it.rel_id("r2")),
              (it.ns_id("n2"), it.rel_id("..."))]
    return it, t6, q, prog, impure


def _cpu_sharded(t6, wildcard, q, gmax, impure):
    """Single-rank run of the protocol over the CPU restatement (test reference)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from keto_amd.sharded import ShardedChecker
    from shard_ref import CpuShardOps
    chk = ShardedChecker(CpuShardOps(t6, wildcard, 0, 1, impure), 0, 1, None, device="cpu", cap=1 << 12,
                         general=False)
    res, err = chk.check(torch.from_numpy(q.view(np.int32).copy()), gmax)
    return res.numpy().copy(), err.numpy().copy()


def _cpu_general_worker(rank, world, port, seed, outq, protocol):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from keto_amd.sharded import ShardedChecker
    from shard_ref import CpuShardOps
    dist_ = None
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist_ = dist
    if seed == "opl":  # every query to the general phase: the gather must cover TTU targets and recursion
        it, t6, q, _, prog = _opl_full_example_graph(7, n_q=600)
        impure = [(a, b) for a in range(it.n_namespaces) for b in range(it.n_relations)]
    else:
        it, t6, q, prog, impure = _impure_graph(seed)
    ops = CpuShardOps(t6, it.wildcard_rel, rank, world, impure, program=prog)
    mine = np.array_split(np.arange(len(q)), world)[rank]
    chk = ShardedChecker(ops, rank, world, dist_, device="cpu", cap=1 << 12, protocol=protocol)
    out = {}
    for gmax in (2, 5):
        res, err = chk.check(torch.from_numpy(q[mine].view(np.int32).copy()), gmax)
        out[gmax] = (mine, res.numpy().copy(), err.numpy().copy())
    outq.put((rank, out, chk.general_queries, chk.general_rows))
    if dist_:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,protocol,seed", [(1, "auto", 5), (2, "dynamic", 5), (2, "fixed", 5), (3, "fixed", 5),
                                                (2, "fixed", "opl"), (3, "dynamic", "opl")])
def test_sharded_general_rewrites_gloo(world, protocol, seed):
    """Queries that reach a rewrite the level protocol cannot evaluate across ranks (here a computed
    rewrite and undeclared relations) are not left as NOT_IMPLEMENTED: every rank gathers the rows of
    the objects its open queries can reach (keto_amd.sharded._gather_region: all-to-all of object
    requests to their owners, rows back to the home rank, gdepth + 1 subject-set hops) and evaluates
    them on that region.  Answers AND error codes equal the oracle's on the whole graph, with the
    oracle program (rewrites, RELATION_NOT_FOUND for undeclared relations)."""
    from oracle.oracle import POLICY_CANONICAL, Oracle
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cpu_general_worker, args=(r, world, port, seed, outq, protocol)) for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    if seed == "opl":
        it, t6, q, _, prog = _opl_full_example_graph(7, n_q=600)
    else:
        it, t6, q, prog, impure = _impure_graph(seed)
    o = Oracle(t6, it.wildcard_rel, prog)
    assert sum(g[2] for g in got) > 0 and sum(g[3] for g in got) > 0  # the general phase ran, rows moved
    for gmax in (2, 5):
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
        res = np.zeros(len(q), np.uint8)
        err = np.zeros(len(q), np.int64)
        for _, out, _, _ in got:
            mine, r, e = out[gmax]
            res[mine], err[mine] = r, e
        bad = np.nonzero((res != exp) | (err != oerr))[0]
        assert bad.size == 0, [(q[i].tolist(), int(res[i]), int(exp[i]), int(err[i]), int(oerr[i])) for i in bad[:8]]
        assert (exp == 1).any() and (exp == 0).any()


def test_sharded_impure_reference_semantics():
    """CPU restatement: queries that reach a rewrite / undeclared relation end as NOT_IMPLEMENTED
    errors; every other query agrees with the oracle on the same graph (which evaluates rewrites)."""
    from oracle.oracle import POLICY_CANONICAL, Oracle
    it, t6, q, prog, impure = _impure_graph(5)
    o = Oracle(t6, it.wildcard_rel, prog)
    n_err = 0
    for gmax in (2, 5):
        res, err = _cpu_sharded(t6, it.wildcard_rel, q, gmax, impure)
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
        ok = err == 0
        assert (res[~ok] == 2).all() and (err[~ok] == 2).all()
        assert (res[ok] == exp[ok]).all() and (oerr[ok] == 0).all()
        n_err += int((~ok).sum())
    assert 0 < n_err


@pytest.mark.gpu
@pytest.mark.parametrize("mat", [0, 1])
def test_sharded_hip_impure_matches_reference(mat, monkeypatch):
    """HIP sharded mode with a rewrite program.  mat = 0 (no materialisation): the NOT_IMPLEMENTED
    errors (root or reached through a subject set) and all other answers equal the CPU restatement's,
    bit for bit.  mat = 1: n1#r2 = union(r0) is a union node, so its queries are answered (the oracle's
    answers) and only the undeclared relations of n2 still end as NOT_IMPLEMENTED."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import HipShardOps, ShardedChecker
    from oracle.oracle import POLICY_CANONICAL, Oracle
    monkeypatch.setenv("KG_MATERIALIZE", str(mat))
    it, t6, q, prog, impure = _impure_graph(5)
    snap = Snapshot(t6, it, prog, 0, shard=(0, 1))
    chk = ShardedChecker(HipShardOps(snap), 0, 1, None, device="cuda", cap=256, general=False)
    o = Oracle(t6, it.wildcard_rel, prog)
    r2 = (q[:, 0] == it.ns_id("n1")) & (q[:, 2] == it.rel_id("r2"))
    assert r2.any()
    for gmax in (2, 5):
        res, err = chk.check(torch.from_numpy(q.view(np.int32).copy()).cuda(), gmax)
        res, err = res.cpu().numpy(), err.cpu().numpy()
        eres, eerr = _cpu_sharded(t6, it.wildcard_rel, q, gmax, impure)
        assert (eerr != 0).any()
        if not mat:
            assert (res == eres).all() and (err == eerr).all(), gmax
            continue
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
        ok = err == 0
        assert (res[~ok] == 2).all() and (err[~ok] == 2).all()
        bad = np.nonzero(ok & ((res != exp) | (oerr != 0)))[0]
        assert bad.size == 0, [(q[i].tolist(), int(res[i]), int(exp[i]), int(oerr[i])) for i in bad[:8]]
        assert (err <= eerr).all() and (err[r2 & (eerr != 0)] == 0).any()  # the union now answers


def _opl_full_example_graph(seed, n_q=2000):
    """The reference parser's full example (tests/golden/opl_full_example.json: view = (parents.traverse(
    viewers) & parents.traverse(view)) | viewers | owners -- a formula recursive through tuple-to-subject-
    set --, not = !owners, rename = siblings.traverse(edit)) on a random graph over its namespaces."""
    import json
    sys.path.insert(0, ROOT)
    from keto_amd.engine import queries_array
    from keto_amd.ketoapi import RelationTuple
    from keto_amd.mapper import Interner
    from keto_amd.namespace import compile_program, namespace_from_json
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "opl_full_example.json")))
    nss = [namespace_from_json({"name": n, "relations": rels}) for n, rels in sorted(golden.items())]
    it = Interner()
    prog_ref = compile_program(nss, it, lower_ttu=False)
    prog = compile_program(nss, it)
    rng = np.random.default_rng(seed)
    files, folders, groups, users = ([f"f{i}" for i in range(60)], [f"d{i}" for i in range(20)],
                                     [f"g{i}" for i in range(15)], [f"u{i}" for i in range(30)])
    kinds = [lambda: f"File:{rng.choice(files)}#parents@(File:{rng.choice(files)}#...)",
             lambda: f"File:{rng.choice(files)}#parents@(Folder:{rng.choice(folders)}#...)",
             lambda: f"File:{rng.choice(files)}#viewers@{rng.choice(users)}",
             lambda: f"File:{rng.choice(files)}#viewers@(Group:{rng.choice(groups)}#members)",
             lambda: f"File:{rng.choice(files)}#owners@{rng.choice(users)}",
             lambda: f"File:{rng.choice(files)}#siblings@(File:{rng.choice(files)}#...)",
             lambda: f"Folder:{rng.choice(folders)}#viewers@(Group:{rng.choice(groups)}#members)",
             lambda: f"Group:{rng.choice(groups)}#members@{rng.choice(users)}",
             lambda: f"Group:{rng.choice(groups)}#members@(Group:{rng.choice(groups)}#members)"]
    tuples = [RelationTuple.from_string(kinds[rng.integers(len(kinds))]()) for _ in range(700)]
    qs = []
    for _ in range(n_q):
        rel = rng.choice(["view", "edit", "not", "rename", "viewers", "owners", "parents"])
        ns, obj = ("Folder", rng.choice(folders)) if rng.random() < 0.2 else ("File", rng.choice(files))
        subj = rng.choice(users + ["nobody"]) if rng.random() < 0.9 else f"(Group:{rng.choice(groups)}#members)"
        qs.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{subj}"))
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    return it, it.tuples_array(tuples), queries_array(q6, rng.integers(-1, 8, len(qs))), prog, prog_ref


def _general_gpu_worker(rank, world, port, outq, kind, driver="py"):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import HipShardOps, ShardedChecker
    dist_ = None
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)  # two ranks on one GPU: host-staged
        dist_ = dist
    torch.cuda.set_device(0)
    if kind == "opl":
        it, t6, q, prog, _ = _opl_full_example_graph(7)
    elif kind == "order":
        it, t6, q, prog, _ = _order_graph()
    else:
        it, t6, q, prog, _ = _impure_graph(5)
    snap = Snapshot(t6, it, prog, 0, shard=(rank, world))
    mine = np.array_split(np.arange(len(q)), world)[rank]
    chk = _checker(driver, snap, rank, world, dist_)
    out = {}
    for gmax in (2, 5, 8):
        res, err = chk.check(torch.from_numpy(q[mine].view(np.int32).copy()).cuda(), gmax)
        out[gmax] = (mine, res.cpu().numpy(), err.cpu().numpy())
    outq.put((rank, out, chk.general_queries))
    if dist_:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,world,driver", [("impure", 1, "py"), ("opl", 1, "py"), ("opl", 2, "py"),
                                               ("order", 1, "py"), ("order", 2, "py"),
                                               ("impure", 1, "lib-rccl-forced"), ("opl", 1, "lib-rccl-forced"),
                                               ("order", 1, "lib-rccl-forced"), ("opl", 1, "lib"),
                                               ("opl", 2, "lib"), ("order", 2, "lib"), ("impure", 2, "lib")])
def test_sharded_general_rewrites_vs_oracle(kind, world, driver):
    """Every rewrite in the hash-sharded mode: the reference parser's full example (a `view` formula
    recursive through tuple-to-subject-set, `not`, nested traverse) and a program with a computed
    rewrite and undeclared relations.  Queries the level protocol ends as NOT_IMPLEMENTED go to the
    general phase (their rows gathered to the home rank, the single-GPU engine's interpreter on them):
    answers and error codes bit-exact with the oracle evaluating the program as written -- at world 2
    over gloo and at world 1 through the exchange protocol over RCCL; world 1 local-first answers every
    query with the replica tier chain (interpreter included)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.oracle import POLICY_CANONICAL, Oracle
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_general_gpu_worker, args=(r, world, port, outq, kind, driver)) for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=150) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    if kind == "opl":
        it, t6, q, _, prog_ref = _opl_full_example_graph(7)
    elif kind == "order":  # a member one level before an earlier branch's error (done-bitmap pruning off)
        it, t6, q, prog_ref, _ = _order_graph()
    else:
        it, t6, q, prog_ref, _ = _impure_graph(5)
    o = Oracle(t6, it.wildcard_rel, prog_ref)
    if driver != "lib" or world > 1:  # (world 1 local-first: the interpreter answers them, no general phase)
        assert sum(g[2] for g in got) > 0
    for gmax in (2, 5, 8):
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
        res = np.zeros(len(q), np.uint8)
        err = np.zeros(len(q), np.int64)
        for _, out, _ in got:
            mine, r, e = out[gmax]
            res[mine], err[mine] = r, e
        bad = np.nonzero((res != exp) | (err != oerr))[0]
        assert bad.size == 0, [(q[i].tolist(), int(res[i]), int(exp[i]), int(err[i]), int(oerr[i])) for i in bad[:8]]
        assert (exp == 1).any() and ((exp == 0).any() or kind == "order")


# ------------------------------------------------------------------ config C4 generator, sharded
def _synth_worker(rank, world, port, n_tuples, n_q, gmax, backend, outq, preset=0, budget=None, back_budget=None,
                  heavy=None, vis=None, bucket=None, driver="py"):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import HipShardOps, ShardedChecker
    dist_ = None
    torch.cuda.set_device(0)
    if backend is not None:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group(backend, rank=rank, world_size=world)
        dist_ = dist
    snap = Snapshot.synthetic(n_tuples, seed=20250131, shard=(rank, world), preset=preset)
    if budget is not None:
        snap.tune("shard_budget", budget)
    if back_budget is not None:
        snap.tune("shard_back_budget", back_budget)
    if heavy is not None:
        snap.tune("shard_heavy", heavy)
    if vis is not None:  # a per-batch visited table of 2^vis (query, node) keys: overflows, reruns larger
        snap.tune("shard_vis", vis)
    dq = torch.empty((n_q, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 31, n_q, dq.data_ptr()), "kg_synth_queries")
    mine = np.array_split(np.arange(n_q), world)[rank]
    if bucket is not None and driver != "py":  # in-library: the first bucket size of the binding
        snap.tune("shard_bucket", bucket)
    chk = _checker(driver, snap, rank, world, dist_, cap=1 << 14)
    if bucket is not None and driver == "py":  # fixed-bucket protocol: B records per destination, far too few
        chk.bucket = bucket
    mq = dq[mine[0]:mine[-1] + 1].contiguous()
    res0, err0 = chk.check(mq, gmax)  # the first batch grows the buckets to fit (overflow reruns)
    res0, err0 = res0.cpu().numpy(), err0.cpu().numpy()
    s0 = chk.host_syncs
    res, err = chk.check(mq, gmax)
    assert (res.cpu().numpy() == res0).all() and (err.cpu().numpy() == err0).all()  # the rerun batch = a clean one
    outq.put((rank, mine, res.cpu().numpy(), err.cpu().numpy(), chk.levels, chk.host_syncs - s0,
              dq.cpu().numpy() if rank == 0 else None, snap.materialized(), chk.back_levels, dict(chk.reruns),
              getattr(chk, "path", None)))
    if dist_:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend,budget,back_budget,heavy",
                         [(1, None, None, None, None), (1, "nccl", None, None, None),
                          (2, "gloo", None, None, None), (1, None, 8, None, None),
                          (1, "nccl", 8, 64, None), (2, "gloo", 8, 64, None),
                          (1, None, None, None, 256), (2, "gloo", None, None, 256), (1, None, 8, 64, 256),
                          (1, None, None, None, 0), (2, "gloo", None, None, 0), (1, "nccl", None, None, 0)])
def test_sharded_c4_generator_vs_oracle(world, backend, budget, back_budget, heavy):
    """Config C4's generator, hash-sharded: world 1 with every level on the device (no host round
    trip per level), world 1 through torch.distributed over RCCL ("nccl": the metadata and record
    all-to-alls run on device tensors), and world 2 (two ranks on one GPU, gloo).  Against the
    oracle on the whole graph's rows, bit-exact; the synthetic queries only touch rewrite-free nodes.
    Budget 8: most walks escalate to the backward phase (the default budget escalates the hub-heavy
    ones only).  heavy 256 / 0: every set row over 256 edges / every set row goes to the flat
    grid-wide hub kernel (k_shard_heavy's tile map), in the forward and the backward phase."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_synth(world, backend, 300_000, 20_000, 10, preset=0, budget=budget, back_budget=back_budget, heavy=heavy)


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend,driver", [(1, None, "lib-loop"), (1, None, "lib-rccl-forced"),
                                                  (2, "gloo", "lib")])
@pytest.mark.parametrize("budget,back_budget", [(8, 64), (8, None), (2, 16)])
def test_sharded_in_library_escalation_vs_oracle(world, backend, driver, budget, back_budget):
    """the escalation phases inside libketogpu.so (kg_shard_comm.hip).  A query whose
    forward records pass the set-edge budget on a rank is dropped from the forward phase, a backward phase
    from its subject's holders (gdepth levels over all-gathered fixed buckets) answers it, and a query past
    the backward budget too walks forward again from its root without a budget -- the single-GPU
    k_stream4 -> k_back -> grid chain, across shards.  C4's generator, bit-exact with the oracle on the
    whole graph: world 1 in the device loop and through the exchange protocol over RCCL, world 2 over
    gloo; budget 2 / back budget 16 sends most queries through all three phases."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_synth(world, backend, 300_000, 20_000, 10, preset=0, budget=budget, back_budget=back_budget, driver=driver)


@pytest.mark.gpu
@pytest.mark.parametrize("heavy,gmax", [(None, 10), (0, 10), (256, 5), (0, 5)])
def test_sharded_one_rank_levels_vs_oracle(heavy, gmax):
    """The one-rank device level loop with every row / rows over 256 edges through the hub kernel and
    at two global depths, bit-exact with the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_synth(1, None, 300_000, 20_000, gmax, preset=0, heavy=heavy)


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend", [(1, None), (2, "gloo")])
def test_sharded_c3_rewrites_vs_oracle(world, backend):
    """Config C3 (Drive-like graph + folder forest + OPL view / edit / share), hash-sharded: view and
    edit are materialised union nodes on every rank (their merged rows hold the parent folder's union
    node, so a query walks the folder chain across ranks), share = view & !blocked is split into its
    own part and two leaf parts and combined by kg_shard_finish.  Bit-exact with the oracle (which
    evaluates the rewrites), no query left to an error."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_synth(world, backend, 150_000, 6000, 10, preset=1)


def _run_synth(world, backend, n_tuples, n_q, gmax, preset, budget=None, back_budget=None, heavy=None,
               vis=None, bucket=None, driver="py"):
    from keto_amd.engine import Snapshot
    from oracle.oracle import POLICY_CANONICAL, Oracle
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_synth_worker, args=(r, world, port, n_tuples, n_q, gmax, backend, outq, preset, budget,
                                                  back_budget, heavy, vis, bucket, driver))
          for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=110) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    q = [g[6] for g in got if g[6] is not None][0].view(np.uint32)
    full = Snapshot.synthetic(n_tuples, seed=20250131, preset=preset)
    o = Oracle(full.export(), 0, full.program if preset else None)
    exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
    assert (oerr == 0).all()
    res = np.zeros(n_q, np.uint8)
    for rank, mine, r, e, levels, syncs, _, mat, back_levels, reruns, path in got:
        assert (e == 0).all(), (rank, np.nonzero(e)[0][:10])
        res[mine] = r
        if world == 1 and backend is None and driver == "py":
            assert syncs == 1 and levels == gmax  # one host round trip for the whole batch
        if driver != "py" and budget is None:  # in-library, no rerun: the path's host round trips and levels
            want = 0 if (world == 1 and "loop" not in driver and "forced" not in driver) else (
                1 if world == 1 and "loop" in driver else 2)
            assert path == want, (path, want, driver)
            want_syncs, want_levels = LIB_PATH_COST[path](gmax)
            assert syncs == want_syncs, (syncs, levels, path)
            assert (levels == want_levels) if path != 2 else (2 <= levels <= want_levels), (syncs, levels, path)
        if budget is not None and budget <= 8 and not preset:
            assert back_levels > 0  # the backward phase ran
        if preset:
            assert mat["union_nodes"] > 0, mat
        if vis is not None:
            assert reruns[2] >= 1, reruns  # the visited table overflowed and the batch reran
        if bucket is not None:
            assert reruns[1] >= 1, reruns  # a bucket overflowed and the batch reran with bigger ones
    bad = np.nonzero(res != exp)[0]
    assert bad.size == 0, [(q[i].tolist(), int(res[i]), int(exp[i])) for i in bad[:8]]
    assert 0.05 < exp.mean() < 0.95


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend,preset,driver", [(1, None, 0, "lib"), (1, None, 1, "lib"),
                                                         (1, None, 0, "lib-loop"), (1, None, 1, "lib-loop"),
                                                         (1, None, 0, "lib-rccl-forced"),
                                                         (1, None, 1, "lib-rccl-forced"),
                                                         (2, "gloo", 0, "lib"), (2, "gloo", 1, "lib"),
                                                         (1, "gloo", 0, "lib-host"), (1, "gloo", 0, "lib-host-forced")])
def test_sharded_in_library_vs_oracle(world, backend, preset, driver):
    """The hash-sharded batch inside libketogpu.so (kg_shard_comm.hip: one kg_check_batch_device call per
    batch, as a Go host makes it): C4's generator (preset 0) and C3's (preset 1: union nodes across ranks,
    split formulas), bit-exact with the oracle on the whole graph:
      world 1 local-first -- the replica tier chain on the rank's rows (no level protocol, no round trip);
      world 1 "-loop" -- the one-rank device level loop (one round trip, gdepth levels);
      world 1 "-rccl-forced" -- the N > 1 exchange protocol over a real RCCL communicator (self send /
        recv, all-gather, all-reduce: the transport code of an 8-GPU run, on one GPU);
      world 2 over the gloo host transport (two ranks on one GPU) and world 1 "-host-forced";
    the exchange protocol: two host round trips per batch, gdepth + 1 exchanges."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_synth(world, backend, 300_000 if preset == 0 else 150_000, 20_000 if preset == 0 else 6000, 10, preset=preset,
               driver=driver)


@pytest.mark.gpu
@pytest.mark.parametrize("world,backend,vis,bucket", [(1, None, 10, None), (2, "gloo", 10, None),
                                                      (2, "gloo", None, 64), (1, "nccl", 11, None),
                                                      ("lib", None, 10, None), ("lib", None, None, 64),
                                                      ("lib-forced", None, 10, 64), ("lib2", "gloo", 10, 64)])
def test_sharded_visited_overflow_reruns(world, backend, vis, bucket):
    """Regression (round 3: "records left after 10 levels" on C3 sharded, an overflow flag OR-ed into a
    sub-bucket count in kg_shard.hip): a C3-shaped graph with a per-batch (query, node) visited table
    of 2^10 / 2^11 keys overflows it, the batch reruns with a larger table (ShardOverflow), and the
    answers and error codes equal the oracle's -- world 1 in the one-rank device loop and over RCCL,
    world 2 over gloo; and the fixed-bucket protocol with 64-record buckets overflows them and reruns
    with bigger ones (reference semantics: internal/check/engine.go:87-145)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    driver = "py"
    if world in ("lib", "lib2"):  # the same through the in-library batch (kg_shard_comm.hip; world 1: its
        # device level loop -- local-first never builds the per-batch (query, node) table or buckets)
        driver, world = ("lib-loop", 1) if world == "lib" else ("lib", 2)
    elif world == "lib-forced":  # world 1, the exchange protocol over RCCL
        driver, world = "lib-rccl-forced", 1
    _run_synth(world, backend, 150_000, 6000, 10, preset=1, vis=vis, bucket=bucket, driver=driver)


def _meta_worker(rank, world, port, outq, n_tuples, n_q, gmax):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for meta in (1, 0):
        snap = Snapshot.synthetic(n_tuples, seed=20250131, shard=(rank, world))
        snap.tune("shard_remote_meta", meta)  # read when the transport binds (collective)
        dq = torch.empty((n_q, 7), dtype=torch.int32, device="cuda")
        _lib.check(_lib.load().kg_synth_queries(snap.handle, 31, n_q, dq.data_ptr()), "kg_synth_queries")
        mine = np.array_split(np.arange(n_q), world)[rank]
        chk = _checker("lib", snap, rank, world, dist)
        r, e = chk.check(dq[mine[0]:mine[-1] + 1].contiguous(), gmax)
        st = chk.chk.stats()
        out[meta] = (r.cpu().numpy(), e.cpu().numpy(), st["records_sent"], st["records_to_peers"])
        chk.chk.close()
        snap.close()
    outq.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_remote_meta_same_answers_fewer_records():
    """Remote child metadata (round 5, kg_shard_comm.hip comm_setup): the first binding all-reduces every
    owner's (set-row length, row signature) word into the other ranks' adjacency records and node map,
    so a remote child that can neither hit nor expand is never sent.  Two ranks on one GPU over gloo,
    C4's generator: the same answers and error codes with the metadata on and off (the oracle check of
    this configuration is test_sharded_in_library_vs_oracle[2-gloo-0-lib]), and fewer records sent and
    fewer crossing to the other rank with it on."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_meta_worker, args=(r, world, port, outq, 300_000, 20_000, 10)) for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=110) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, out in got:
        (r1, e1, sent1, peers1), (r0, e0, sent0, peers0) = out[1], out[0]
        assert (r1 == r0).all() and (e1 == e0).all(), rank
        assert (e1 == 0).all() and 0.05 < r1.mean() < 0.95
        assert sent1 < sent0 and peers1 < peers0, (rank, sent1, sent0, peers1, peers0)


def _bound_worker(rank, world, port, outq, driver, mode):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    dist_ = None
    torch.cuda.set_device(0)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist_ = dist
    snap = Snapshot.synthetic(150_000, seed=20250131, shard=(rank, world))
    n_q = 8000
    dq = torch.empty((n_q, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 77, n_q, dq.data_ptr()), "kg_synth_queries")
    mine = np.array_split(np.arange(n_q), world)[rank]
    mq = dq[mine[0]:mine[-1] + 1].contiguous()
    snap.tune("shard_bucket", 64)  # far too small: the first run overflows
    if mode == "overflow":  # every run reports a bucket overflow: a persistent one
        snap.tune("shard_force_overflow", 1)
        snap.tune("shard_max_reruns", 3)
    else:  # the bucket the batch needs is over the buffer cap
        snap.tune("shard_max_bytes", 1 << 16)
    chk = _checker(driver, snap, rank, world, dist_)
    t0 = time.time()
    try:
        chk.check(mq, 10)
        outcome = "ok"
    except _lib.KetoGPUError as e:
        outcome = str(e)
    took = time.time() - t0
    # the binding stays usable: the same batch with sane limits
    snap.tune("shard_force_overflow", 0)
    snap.tune("shard_max_bytes", 0)
    res, err = chk.check(mq, 10)
    outq.put((rank, outcome, took, mine, res.cpu().numpy(), err.cpu().numpy(), dq.cpu().numpy() if rank == 0 else None))
    if dist_:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("driver,world", [("lib-loop", 1), ("lib-rccl-forced", 1), ("lib", 2)])
@pytest.mark.parametrize("mode", ["overflow", "bytes"])
def test_sharded_rerun_bound(driver, world, mode):
    """the overflow rerun loop is bounded.  A persistent bucket overflow
    (kg_snapshot_tune shard_force_overflow) ends after shard_max_reruns reruns, and a bucket larger than
    the buffer cap (shard_max_bytes) ends at once -- every rank returns KG_ERR_RESOURCE (-4) together, in
    seconds, with no out-of-memory and no rank left waiting in a collective; the binding then answers the
    same batch bit-exact with the oracle.  World 1 in the device loop and over RCCL (the exchange
    protocol), world 2 over gloo."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from keto_amd.engine import Snapshot
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bound_worker, args=(r, world, port, outq, driver, mode)) for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=110) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    want = "after 3 reruns" if mode == "overflow" else "cap"
    for rank, outcome, took, *_ in got:
        assert "(-4)" in outcome and want in outcome, (rank, outcome)
        assert took < 60, took
    q = [g[6] for g in got if g[6] is not None][0].view(np.uint32)
    full = Snapshot.synthetic(150_000, seed=20250131)
    exp = _expected(full.export(), 0xFFFFFFFF, q, 10)
    res = np.zeros(len(q), np.uint8)
    for _, _, _, mine, r, e, _ in got:
        assert (e == 0).all()
        res[mine] = r
    bad = np.nonzero(res != exp)[0]
    assert bad.size == 0, bad[:8]


def _nodict_graph():
    """Rows in a relation no dict and no program names (the dict is NULL, so the snapshot's relation count
    comes from the program): n1:b#zz@u1 decides n1:a#r2@u1 (r2 = computed r0, r0 -> (n1:b#zz)) through
    checkDirect before astRelationFor's error for the undeclared zz (engine.go:183-207) -- only when the
    general phase's region gather brings the zz rows (gather_region asked for relations
    [0, n_rel) only)."""
    sys.path.insert(0, ROOT)
    from keto_amd.engine import queries_array
    from keto_amd.ketoapi import RelationTuple
    from keto_amd.mapper import Interner
    from keto_amd.namespace import ComputedSubjectSet, Namespace, Relation, SubjectSetRewrite, compile_program
    it = Interner()
    nss = [Namespace("n1", [Relation("r0"), Relation("r1"), Relation("r2", rewrite=SubjectSetRewrite([
        ComputedSubjectSet("r0")]))])]
    prog = compile_program(nss, it)
    rows = []
    for i in range(40):
        rows += [f"n1:a{i}#r0@(n1:b{i}#zz)", f"n1:b{i}#zz@u{i % 7}", f"n1:a{i}#r1@u{(i + 1) % 7}",
                 f"n1:c{i}#r0@(n1:a{(i + 3) % 40}#r2)"]
    tuples = [RelationTuple.from_string(x) for x in rows]
    t6 = it.tuples_array(tuples)
    assert it.rel_id("zz") > max(it.rel_id(r) for r in ("r0", "r1", "r2"))
    qs = []
    for i in range(40):
        for u in range(8):
            for rel, obj in (("r2", "a"), ("r0", "c"), ("r0", "a")):
                qs.append(RelationTuple.from_string(f"n1:{obj}{i}#{rel}@u{u}"))
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    return it, t6, queries_array(q6, np.zeros(len(qs), np.int64)), prog


def _nodict_worker(rank, world, port, outq, driver):
    sys.path.insert(0, ROOT)
    import ctypes as C
    import torch.distributed as dist
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    dist_ = None
    torch.cuda.set_device(0)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist_ = dist
    it, t6, q, prog = _nodict_graph()
    L = _lib.load()
    holder = Snapshot(None, it, prog, 0, _handle=C.c_void_p(), shard=(rank, world))
    pc = holder._prog(prog)
    t = np.ascontiguousarray(t6, np.uint32)
    h = C.c_void_p()
    _lib.check(L.kg_snapshot_create_shard(t.ctypes.data_as(C.c_void_p), t.shape[0], None, C.byref(pc), 0, rank, world,
                                          C.byref(h)), "kg_snapshot_create_shard (NULL dict)")
    holder._h = h
    mine = np.array_split(np.arange(len(q)), world)[rank]
    chk = _checker(driver, holder, rank, world, dist_)
    out = {}
    for gmax in (3, 6):
        res, err = chk.check(torch.from_numpy(q[mine].view(np.int32).copy()).cuda(), gmax)
        out[gmax] = (mine, res.cpu().numpy(), err.cpu().numpy())
    outq.put((rank, out, chk.general_queries))
    if dist_:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,driver", [(1, "lib-rccl-forced"), (2, "lib"), (1, "lib")])
def test_sharded_general_phase_null_dict(world, driver):
    """a snapshot created with a NULL dict whose rows use a relation the program never
    names.  The general phase gathers every relation's rows of an object (rel_span: 1 + the largest
    relation id of any node), so the answers and error codes equal the oracle's on the program as
    written; world 1 local-first answers without any gather."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.oracle import POLICY_CANONICAL, Oracle
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_nodict_worker, args=(r, world, port, outq, driver)) for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=110) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    it, t6, q, prog = _nodict_graph()
    o = Oracle(t6, 0xFFFFFFFF, prog)
    if driver != "lib" or world > 1:
        assert sum(g[2] for g in got) > 0  # the general phase answered some
    for gmax in (3, 6):
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
        res = np.zeros(len(q), np.uint8)
        err = np.zeros(len(q), np.int64)
        for _, out, _ in got:
            mine, r, e = out[gmax]
            res[mine], err[mine] = r, e
        bad = np.nonzero((res != exp) | (err != oerr))[0]
        assert bad.size == 0, [(q[i].tolist(), int(res[i]), int(exp[i]), int(err[i]), int(oerr[i])) for i in bad[:8]]
        assert (exp == 1).any() and (oerr != 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("sharded", [False, True])
def test_formula_ttu_leaves_vs_oracle(sharded):
    """Boolean rewrites with tuple-to-subject-set leaves (rewrites.go:205-260 inside binop.go's and / or
    and rewrites.go:95-159's not): lowered to hidden union relations (namespace.lower_ttu_leaves), they
    are materialised and split like computed leaves -- on one GPU without the interpreter, and in the
    hash-sharded mode (world 1, on the device) without KG_ERR_NOT_IMPLEMENTED.  Bit-exact with the
    oracle evaluating the program as written."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, ROOT)
    from keto_amd.engine import Config, Engine, Snapshot, queries_array
    from keto_amd.ketoapi import RelationTuple
    from keto_amd.mapper import Interner
    from keto_amd.namespace import (ComputedSubjectSet as Cm, InvertResult as Nt, Namespace, Relation,
                                    SubjectSetRewrite as Or, TupleToSubjectSet as Tt, compile_program)
    from keto_amd.sharded import HipShardOps, ShardedChecker
    from oracle.oracle import POLICY_CANONICAL, Oracle
    rng = np.random.default_rng(4242)
    rels = [Relation("a"), Relation("b"), Relation("parent"),
            Relation("u1", rewrite=Or([Cm("a"), Tt("parent", "u1")])),
            Relation("g", rewrite=Or([Cm("a"), Tt("parent", "u1")], "and")),
            Relation("h", rewrite=Or([Cm("b"), Nt(Tt("parent", "a"))])),
            Relation("k", rewrite=Or([Or([Tt("parent", "b"), Cm("u1")], "and"), Nt(Cm("b"))], "and"))]
    nss = [Namespace("d", rels)]
    it = Interner()
    prog_ref = compile_program(nss, it, lower_ttu=False)
    n_obj, n_users = 80, 25
    tuples = []
    for _ in range(900):
        x = f"d:o{rng.integers(n_obj)}"
        r = rng.random()
        if r < 0.3:
            tuples.append(f"{x}#parent@(d:o{rng.integers(n_obj)}#...)")
        elif r < 0.8:
            tuples.append(f"{x}#{'a' if rng.random() < 0.6 else 'b'}@u{rng.integers(n_users)}")
        else:  # subject sets of a plain relation (a set edge into a u1 node of an object without u1
            # rows would reach an unmaterialised rewrite: the interpreter's case, an error when sharded)
            tuples.append(f"{x}#a@(d:o{rng.integers(n_obj)}#a)")
    tuples = [RelationTuple.from_string(t) for t in tuples]
    t6 = it.tuples_array(tuples)
    prog = compile_program(nss, it)
    qs = [RelationTuple.from_string(f"d:o{rng.integers(n_obj)}#{rng.choice(['g', 'h', 'k', 'u1'])}@u{rng.integers(n_users)}")
          for _ in range(3000)]
    q6 = np.asarray([it.tuple_ids(t) for t in qs], np.uint32)
    depths = rng.integers(0, 7, len(qs))
    oracle = Oracle(t6, it.wildcard_rel, prog_ref)
    if sharded:
        snap = Snapshot(t6, it, prog, 0, shard=(0, 1))
        chk = ShardedChecker(HipShardOps(snap), 0, 1, None, device="cuda", cap=1 << 12)
    else:
        snap = Snapshot(t6, it, prog, 0)
    q7 = queries_array(q6, depths)
    for gmax in (2, 4, 6):
        if sharded:
            res, err = chk.check(torch.from_numpy(q7.view(np.int32).copy()).cuda(), gmax)
            out, err = res.cpu().numpy(), err.cpu().numpy()
        else:
            e = Engine(snap, Config(gmax))
            out, err = e.batch_check_ids(q7, with_stats=True)
            assert e.last_stats["n_general"] == 0, e.last_stats  # split, not interpreted
        exp, oerr, _ = oracle.check_batch(q6, depths, gmax, POLICY_CANONICAL)
        bad = np.nonzero((out != exp) | (err.astype(np.int64) != oerr))[0]
        assert bad.size == 0, [(str(qs[i]), int(depths[i]), int(out[i]), int(exp[i]), int(err[i])) for i in bad[:8]]
        assert 0.05 < (out == 1).mean() < 0.95 and (oerr == 0).all()


def _order_graph():
    """A member found at a shallow level in a LATER branch, an error deeper in an EARLIER one:
    d:x#a has rows (d:y#a), (d:z#a) in that order; d:y#a -> (d:w#nope) where nope is undeclared
    (checkIsAllowed on it fails with RELATION_NOT_FOUND, engine.go:228); d:z#a holds u directly.
    The canonical recursion visits y's subtree first, so x#a@u is an error at every depth >= 2 (w's
    relation is looked up even at rest depth 0), although z's direct tuple is found one level
    before w is reached."""
    sys.path.insert(0, ROOT)
    from keto_amd.engine import queries_array
    from keto_amd.ketoapi import RelationTuple
    from keto_amd.mapper import Interner
    from keto_amd.namespace import Namespace, Relation, compile_program
    it = Interner()
    rows = ["d:x#a@(d:y#a)", "d:x#a@(d:z#a)", "d:y#a@(d:w#nope)", "d:z#a@u", "d:w#nope@v", "d:p#a@(d:x#a)"]
    t6 = it.tuples_array([RelationTuple.from_string(r) for r in rows])
    prog = compile_program([Namespace("d", [Relation("a")])], it)
    qs = ["d:x#a@u", "d:p#a@u", "d:z#a@u", "d:y#a@u", "d:x#a@v"]
    q6 = np.asarray([it.tuple_ids(RelationTuple.from_string(x)) for x in qs], np.uint32)
    q = np.concatenate([queries_array(q6, d) for d in (2, 3, 4, 5)])
    impure = [(it.ns_id("d"), it.rel_id("nope"))]
    return it, t6, q, prog, impure


@pytest.mark.parametrize("general", [True, False])
def test_sharded_member_does_not_hide_an_earlier_error(general):
    """The level protocol finds z's direct tuple one level before it reaches w's undeclared relation;
    pruning the query's records once it is a member would hide the error the canonical order
    reports first.  With errors possible in the graph the protocol does not prune, so the query ends
    NOT_IMPLEMENTED and the general phase gives the oracle's answer (general off: the error stays)."""
    from oracle.oracle import POLICY_CANONICAL, Oracle
    from keto_amd.sharded import ShardedChecker
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from shard_ref import CpuShardOps
    it, t6, q, prog, impure = _order_graph()
    o = Oracle(t6, it.wildcard_rel, prog)
    for gmax in (2, 5):
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL)
        chk = ShardedChecker(CpuShardOps(t6, it.wildcard_rel, 0, 1, impure, program=prog), 0, 1, None, device="cpu",
                             cap=1 << 10, general=general)
        res, err = chk.check(torch.from_numpy(q.view(np.int32).copy()), gmax)
        res, err = res.numpy(), err.numpy()
        if general:
            assert (res == exp).all() and (err == oerr).all(), (gmax, res, exp, err, oerr)
        else:  # every query the oracle answers with an error is an error here too (never a member)
            assert (res[oerr != 0] == 2).all(), (gmax, res, exp, err, oerr)
    assert (oerr != 0).any() and (exp == 1).any()


# ------------------------------------------------------------------ expand on a hash-sharded snapshot
def _expand_graph(seed):
    sys.path.insert(0, ROOT)
    from keto_amd.ketoapi import RelationTuple
    from keto_amd.mapper import SUBJECT_ID, Interner
    rng = np.random.default_rng(seed)
    n_obj = 70
    tuples = []
    for _ in range(900):
        ns, obj, rel = rng.choice(["a", "b"]), f"o{rng.integers(n_obj)}", rng.choice(["r0", "r1", "r2"])
        if rng.random() < 0.55:
            s = f"({rng.choice(['a', 'b'])}:o{rng.integers(n_obj)}#{rng.choice(['r0', 'r1', 'r2', '...'])})"
        else:
            s = f"u{rng.integers(30)}"
        tuples.append(RelationTuple.from_string(f"{ns}:{obj}#{rel}@{s}"))
    it = Interner()
    t6 = it.tuples_array(tuples)
    roots = []
    for _ in range(300):
        if rng.random() < 0.05:
            roots.append([SUBJECT_ID, it.obj_id(f"u{rng.integers(30)}"), 0, 0])
        else:
            roots.append([it.ns_id(rng.choice(["a", "b"])), it.obj_id(f"o{rng.integers(n_obj + 2)}"),
                          it.rel_id(rng.choice(["r0", "r1", "r2"])), int(rng.integers(-1, 7)) & 0xFFFFFFFF])
    return it, t6, np.asarray(roots, np.uint32)


def _expand_worker(rank, world, port, transport, outq):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from keto_amd.engine import Snapshot
    from keto_amd.sharded import LibShardedChecker
    dist_ = None
    if transport == "host":
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist_ = dist
    torch.cuda.set_device(0)
    it, t6, roots = _expand_graph(5)
    snap = Snapshot(t6, it, None, 0, shard=(rank, world))
    chk = LibShardedChecker(snap, rank, world, dist_, transport=transport, snapshot_stream=True)
    mine = np.array_split(np.arange(len(roots)), world)[rank]
    out = {}
    for gmax in (1, 3, 6):
        out[gmax] = (mine, chk.expand(roots[mine], gmax))
    outq.put((rank, out))
    if dist_:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,transport", [(1, "rccl"), (2, "host"), (3, "host")])
def test_sharded_expand_vs_oracle(world, transport):
    """kg_expand_batch on a hash-sharded snapshot (collective; the rows the roots can reach gathered to
    their rank, then the single-GPU BuildTree, internal/expand/engine.go:35-104): every tree equals the
    oracle's on the whole graph record for record (same pre-order, same child order) -- world 1 over RCCL,
    worlds 2 and 3 over the gloo host transport."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.oracle import Oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_expand import _cmp_records
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_expand_worker, args=(r, world, port, transport, outq)) for r in range(world)]
    for p in ps:
        p.start()
    got = [outq.get(timeout=150) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    it, t6, roots = _expand_graph(5)
    oracle = Oracle(t6, it.wildcard_rel)
    n_trees = 0
    for _, out in got:
        for gmax, (mine, trees) in out.items():
            for i, g in zip(mine, trees):
                r = roots[i]
                exp = oracle.expand(int(r[0]), int(r[1]), int(r[2]), int(np.uint32(r[3]).view(np.int32)), gmax)
                _cmp_records(exp, g, (r.tolist(), gmax))
                n_trees += g is not None
    assert n_trees > 100


def _learned_worker(outq, n_tuples, n_q):
    sys.path.insert(0, ROOT)
    from keto_amd import _lib
    from keto_amd.engine import Snapshot
    torch.cuda.set_device(0)
    snap = Snapshot.synthetic(n_tuples, seed=20250131, shard=(0, 1))
    dq = torch.empty((n_q, 7), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().kg_synth_queries(snap.handle, 77, n_q, dq.data_ptr()), "kg_synth_queries")
    chk = _checker("lib-rccl-forced", snap, 0, 1, None, cap=1 << 14)
    out = []
    for gmax in (3, 3, 10, 10):  # a shallow batch teaches few exchanges; the deep one after it reruns
        r, e = chk.check(dq, gmax)
        st = chk.chk.stats()
        out.append((gmax, r.cpu().numpy(), e.cpu().numpy(), st["exchanges"], st["exchange_reruns"]))
    outq.put((dq.cpu().numpy(), out))


@pytest.mark.gpu
def test_sharded_learned_exchanges_rerun():
    """The exchange protocol runs the number of exchanges the previous batch needed (its last non-empty
    one + 2) instead of gdepth + 1.  A gdepth-3 batch learns <= 4; the gdepth-10
    batch after it has records left after them and reruns with all 11 exchanges, then the next one runs
    the learned count with no rerun -- every answer equal to the oracle's (world 1 over RCCL, forced)."""
    from keto_amd.engine import Snapshot
    from oracle.oracle import POLICY_CANONICAL, Oracle
    ctx = mp.get_context("spawn")
    outq = ctx.Queue()
    p = ctx.Process(target=_learned_worker, args=(outq, 300_000, 20_000))
    p.start()
    dq, out = outq.get(timeout=110)
    p.join(60)
    assert p.exitcode == 0
    q = dq.view(np.uint32)
    full = Snapshot.synthetic(300_000, seed=20250131)
    o = Oracle(full.export(), 0)
    for k, (gmax, r, e, xch, reruns) in enumerate(out):
        exp, oerr, _ = o.check_batch(q[:, :6], q[:, 6].view(np.int32), gmax, POLICY_CANONICAL, nthreads=8)
        assert (e == 0).all() and (r == exp).all(), (k, gmax, np.nonzero(r != exp)[0][:8])
        assert xch <= gmax + 1, (k, xch)
    assert out[2][4] == 1 and out[2][3] == 11, out[2][3:]  # records left after the learned count: one rerun
    assert out[3][4] == 0 and out[3][3] <= 11, out[3][3:]  # learned from the deep batch: no rerun
