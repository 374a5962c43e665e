"""OPL front end (keto_amd/opl.py) against the reference's own parser and lexer fixtures
(internal/schema/parser_test.go, lexer_test.go and their .snapshots, transcribed by
tests/golden/make_opl_golden.py), plus the parser's documented limits and quirks."""
import json
import os

import pytest

from keto_amd import opl
from keto_amd.namespace import (ComputedSubjectSet, InvertResult, SubjectSetRewrite, child_to_json,
                                compile_program, namespace_to_json)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _ast(nss):
    return {n.name: namespace_to_json(n).get("relations", []) for n in nss}


def test_full_example_matches_reference_snapshot():
    text = open(os.path.join(GOLDEN, "opl_full_example.opl")).read()
    nss, errs = opl.parse(text)
    assert errs == []
    assert _ast(nss) == json.load(open(os.path.join(GOLDEN, "opl_full_example.json")))


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLDEN, "opl_lexer.json")))["lexable"],
                         ids=lambda c: c["name"])
def test_lexer_snapshots(case):
    assert [str(i) for i in opl.lex(case["input"])] == case["tokens"]


@pytest.mark.parametrize("case", json.load(open(os.path.join(GOLDEN, "opl_lexer.json")))["errors"],
                         ids=lambda c: c["name"])
def test_lexer_errors(case):
    assert opl.lex(case["input"])[-1].typ == opl.ERROR


def test_parser_error_unclosed_comment():  # parser_test.go:12-14
    _, errs = opl.parse("/* unclosed comment")
    assert errs


def _perm(expr):
    return "class N implements Namespace { related: { a: N[]  b: N[]  c: N[] } permits = { p: (ctx: Context) => %s } }" % expr


def _rewrite(expr):
    nss, errs = opl.parse(_perm(expr))
    assert errs == [], [str(e) for e in errs]
    return child_to_json([r for r in nss[0].relations if r.name == "p"][0].rewrite)


A = "this.related.a.includes(ctx.subject)"
B = "this.related.b.includes(ctx.subject)"
C = "this.related.c.includes(ctx.subject)"


def _or(*c):
    return {"operator": "or", "children": list(c)}


def _and(*c):
    return {"operator": "and", "children": list(c)}


a, b, c = {"relation": "a"}, {"relation": "b"}, {"relation": "c"}


def test_left_assoc_no_precedence():
    # a || b && c == (a || b) && c (parser.go:317-324): an operator makes the tree so far its first
    # child, and a single expression is wrapped in "or" (AsRewrite); simplifyExpression merges only
    # same-operator children of the ROOT chain, so the inner single-child "or" survives (as in the
    # reference's full_example snapshot)
    assert _rewrite(f"{A} || {B} && {C}") == _and(_or(_or(a), b), c)
    assert _rewrite(f"{A} || {B} || {C}") == _or(a, b, c)
    assert _rewrite(f"{A} && {B} && {C}") == _and(_or(a), b, c)


def test_not_and_groups():
    assert _rewrite(f"!{A}") == _or({"inverted": a})
    assert _rewrite(f"!({A} && {B})") == _or({"inverted": _and(_or(a), b)})
    assert _rewrite(f"{A} && ({B} || {C})") == _and(_or(a), _or(_or(b), c))


def test_traverse_forms():
    rw = _rewrite("this.related.a.traverse((x) => x.related.b.includes(ctx.subject)) || "
                  "this.related.a.traverse(x => x.permits.p(ctx))")
    assert rw == {"operator": "or", "children": [{"relation": "a", "computed_subject_set_relation": "b"},
                                                 {"relation": "a", "computed_subject_set_relation": "p"}]}


def test_nesting_limit():
    deep = "(" * 10 + A + ")" * 10
    _, errs = opl.parse(_perm(deep))
    assert errs and "nested too deeply" in errs[0].msg
    ok = "(" * 9 + A + ")" * 9
    assert opl.parse(_perm(ok))[1] == []


def test_typecheck_errors():
    _, errs = opl.parse("class N implements Namespace { related: { a: Nope[] } permits = { "
                        "p: (ctx: Context) => this.related.zz.includes(ctx.subject) } }")
    msgs = [e.msg for e in errs]
    assert any("namespace 'Nope' was not declared" in m for m in msgs)
    assert any("did not declare relation 'zz'" in m for m in msgs)


def test_two_expressions_in_a_row_are_siblings():
    # the reference keeps expecting an expression after one (parser.go:349): both become children
    assert _rewrite(f"{A} {B}") == {"operator": "or", "children": [{"relation": "a"}, {"relation": "b"}]}


def _norm(j):
    """Drops single-child "or" nodes below the root: the same 3-valued result (binop.go:15-45)."""
    if "children" in j:
        kids = [_norm(x) for x in j["children"]]
        kids = [k["children"][0] if ("children" in k and k["operator"] == "or" and len(k["children"]) == 1) else k
                for k in kids]
        return {"operator": j["operator"], "children": kids}
    if "inverted" in j:
        return {"inverted": _norm(j["inverted"])}
    return j


def test_c3_namespace_in_opl_matches_the_synthetic_namespaces():
    """Config C3's namespaces written in OPL: the same relations, and rewrites equal to the ones
    keto_amd.synth builds up to the parser's single-child "or" wrappers."""
    from keto_amd import synth
    got = {n.name: namespace_to_json(n).get("relations", []) for n in opl.parse_strict(synth.C3_OPL)}
    want = {n.name: namespace_to_json(n).get("relations", []) for n in synth.c3_namespaces()}
    assert got.pop("user") == []
    assert set(got) == set(want)
    for ns in want:
        assert [r["name"] for r in got[ns]] == [r["name"] for r in want[ns]], ns
        for g, w in zip(got[ns], want[ns]):
            assert ("rewrite" in g) == ("rewrite" in w)
            if "rewrite" in g:
                assert _norm(g["rewrite"]) == _norm(w["rewrite"]), (ns, g["name"])
