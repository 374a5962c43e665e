"""The CPU oracle against every golden vector of the reference's own tests."""
import pytest

from golden_cases import Case, all_cases
from keto_amd.ketoapi import trees_equal_unordered
from oracle.oracle import POLICY_CANONICAL, POLICY_DFS, Oracle, records_to_tree

CHECK_CASES = all_cases("checks")
EXPAND_CASES = all_cases("expands")


@pytest.mark.parametrize("fn,case", CHECK_CASES, ids=[f"{f}:{c['name']}" for f, c in CHECK_CASES])
@pytest.mark.parametrize("policy", [POLICY_CANONICAL, POLICY_DFS], ids=["canonical", "dfs"])
def test_oracle_checks(fn, case, policy):
    c = Case(case)
    o = Oracle(c.arr, c.it.wildcard_rel, c.prog)
    for chk in case["checks"]:
        r, err = o.check(c.query(chk["tuple"]), chk["max_depth"], chk["global_max_depth"], policy)
        assert err == 0, chk
        assert r == int(chk["allowed"]), (chk, r)


@pytest.mark.parametrize("fn,case", EXPAND_CASES, ids=[f"{f}:{c['name']}" for f, c in EXPAND_CASES])
def test_oracle_expand(fn, case):
    c = Case(case)
    o = Oracle(c.arr, c.it.wildcard_rel, c.prog)
    for e in case["expands"]:
        rec = o.expand(*c.expand_root(e), e["max_depth"], e["global_max_depth"])
        got = records_to_tree(rec, c.it)
        exp = Case.expected_tree(e)
        if e.get("ordered"):
            assert got == exp
        else:
            assert trees_equal_unordered(got, exp), (got, exp)


@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_expand_nodes_batch(threads):
    """ko_expand_nodes_batch (the C5 CPU baseline) builds the same trees as ko_expand_node, root by root,
    including a tree larger than a worker's first buffer (70 k records: the grow-and-rebuild path)."""
    import numpy as np
    SET = 0x80000000
    rng = np.random.default_rng(3)
    n = 400
    rows = [[] for _ in range(n)]
    for v in range(n - 1):
        for _ in range(int(rng.integers(0, 6))):
            c = int(rng.integers(0, n - 1))
            rows[v].append(SET | c if rng.random() < 0.6 else 1000 + c)
    rows[n - 1] = [5000 + i for i in range(70000)]  # one wide row: 70 001 records at depth >= 2
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in rows])
    subj = np.array([s for r in rows for s in r], np.uint32)
    nd = np.arange(n, dtype=np.uint32)
    o = Oracle.from_csr(0, np.zeros(n, np.uint32), nd, np.ones(n, np.uint32), off, subj)
    nodes = np.concatenate([np.arange(n, dtype=np.uint32), [n - 1, 7]]).astype(np.uint32)
    depths = np.array([int(x) % 6 for x in range(len(nodes))], np.int32)
    got = o.expand_nodes_batch(nodes, depths, 5, threads)
    for i, (v, d) in enumerate(zip(nodes, depths)):
        rec = o.expand_node(int(v), int(d), 5)
        assert got[i] == (0 if rec is None else len(rec)), (i, v, d)
    assert got.max() == 70001
