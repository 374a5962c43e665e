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
