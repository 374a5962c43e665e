"""Handler semantics (keto_amd/handlers.py): request decoding on the CPU; status mirroring, the
unknown-namespace rule and the expand responses through the HIP engines (-m gpu)."""
import pytest

from keto_amd.handlers import (CheckHandler, ExpandHandler, HandlerError, max_depth_from_query, parse_go_int,
                               parse_query, tuple_from_json, tuple_from_url_query)
from keto_amd.ketoapi import RelationTuple, SubjectSet


def test_parse_go_int():
    # strconv.ParseInt(s, 0, 0)
    for s, v in [("0", 0), ("5", 5), ("-3", -3), ("+7", 7), ("010", 8), ("0x1F", 31), ("0b101", 5), ("0o17", 15),
                 ("1_000", None), ("0x_1F", 31), ("9223372036854775807", 2 ** 63 - 1)]:
        if v is None:
            with pytest.raises(ValueError):
                parse_go_int(s)
        else:
            assert parse_go_int(s) == v, s
    for s in ["", "abc", "1.5", "08", "0x", "9223372036854775808", "1__0", " 1"]:
        with pytest.raises(ValueError):
            parse_go_int(s)


def test_max_depth_query():
    assert max_depth_from_query(parse_query("")) == 0  # absent: the global default
    assert max_depth_from_query(parse_query("max-depth=3")) == 3
    with pytest.raises(HandlerError) as e:
        max_depth_from_query(parse_query("max-depth=three"))
    assert e.value.status == 400


def test_tuple_from_url_query():
    t = tuple_from_url_query(parse_query("namespace=n&object=o&relation=r&subject_id=u"))
    assert t == RelationTuple("n", "o", "r", subject_id="u")
    t = tuple_from_url_query(parse_query("namespace=n&object=o&relation=r&subject_set.namespace=g&"
                                         "subject_set.object=x&subject_set.relation=m"))
    assert t.subject_set == SubjectSet("g", "x", "m")
    # ketoapi/public_api_definitions.go:15-19
    for q, frag in [("namespace=n&object=o&relation=r&subject=u", "dropped"),
                    ("namespace=n&object=o&relation=r&subject_id=u&subject_set.namespace=g", "exactly one"),
                    ("namespace=n&object=o&relation=r&subject_set.namespace=g", "incomplete subject"),
                    ("namespace=n&object=o&relation=r", "nil"),
                    ("namespace=n&relation=r&subject_id=u", "incomplete tuple")]:
        with pytest.raises(HandlerError) as e:
            tuple_from_url_query(parse_query(q))
        assert e.value.status == 400 and frag in e.value.message, q


def test_tuple_from_json():
    t = tuple_from_json(b'{"namespace":"n","object":"o","relation":"r","subject_id":"u"}')
    assert t == RelationTuple("n", "o", "r", subject_id="u")
    with pytest.raises(HandlerError) as e:
        tuple_from_json(b"{not json")
    assert e.value.status == 400 and "could not unmarshal json" in e.value.message


@pytest.mark.gpu
def test_check_handler_mirroring_and_unknown_namespace():
    """REST 200/403 mirroring, /openapi always 200, unknown namespace -> false over REST and an error
    over gRPC, engine errors -> 500 (handler.go:101-275)."""
    from golden_cases import Case, all_cases
    from keto_amd.engine import Registry
    fn, case = [x for x in all_cases("checks") if x[0] == "rewrites_test.json"][0]
    c = Case(case)
    reg = Registry(c.tuples, c.namespaces, interner=c.it)
    h = CheckHandler(reg.permission_engine(), reg.mapper)
    ok = "namespace=doc&object=document&relation=owner&subject_id=user"
    no = "namespace=doc&object=document&relation=owner&subject_id=nobody"
    unknown = "namespace=nope&object=document&relation=owner&subject_id=user"
    assert h.get_check(ok) == (200, {"allowed": True})
    assert h.get_check(no) == (403, {"allowed": False})
    assert h.get_check(no, mirror_status=False) == (200, {"allowed": False})
    assert h.get_check(unknown) == (403, {"allowed": False})
    assert h.get_check(unknown, mirror_status=False) == (200, {"allowed": False})
    assert h.post_check({"namespace": "doc", "object": "document", "relation": "owner", "subject_id": "user"}) == \
        (200, {"allowed": True})
    assert h.post_check(b'{"namespace":"nope","object":"x","relation":"y","subject_id":"u"}') == \
        (403, {"allowed": False})
    assert h.get_check(ok + "&max-depth=abc")[0] == 400
    assert h.get_check("namespace=doc&object=document&relation=owner")[0] == 400
    # an undeclared relation of a configured namespace: engine error -> 500
    st, body = h.get_check("namespace=doc&object=document&relation=undeclared&subject_id=user")
    assert st == 500 and "relation not found" in body["error"]["message"]
    # gRPC: the tuple field wins over the deprecated flat fields; unknown namespace is an error
    r = h.grpc_check({"tuple": {"namespace": "doc", "object": "document", "relation": "viewer",
                                "subject": {"id": "user"}},
                      "namespace": "nope", "max_depth": 0})
    assert r == {"allowed": True, "snaptoken": "not yet implemented"}
    with pytest.raises(HandlerError) as e:
        h.grpc_check({"tuple": {"namespace": "nope", "object": "x", "relation": "y", "subject": {"id": "u"}}})
    assert e.value.status == 404 and e.value.grpc_code == 5


@pytest.mark.gpu
def test_expand_handler_responses():
    """gRPC: a subject id is a leaf of itself, a nil tree an empty response (expand/handler.go:109-146);
    REST: the tree JSON, 404 for an unknown namespace."""
    from golden_cases import Case, all_cases
    from keto_amd.engine import Registry
    from keto_amd.ketoapi import Tree, trees_equal_unordered
    cases = {c["name"]: c for _, c in all_cases("expands")}
    for name in ("expand handler returns tree", "unknown subject set expands to nil"):
        case = cases[name]
        c = Case(case)
        reg = Registry(c.tuples, c.namespaces, interner=c.it)
        h = ExpandHandler(reg.expand_engine(), reg.mapper)
        assert h.grpc_expand({"subject": {"id": "u1"}}) == {"tree": {"node_type": "leaf", "subject": {"id": "u1"}}}
        e = case["expands"][0]
        ss = e["subject_set"]
        got = h.grpc_expand({"subject": {"set": ss}, "max_depth": e["max_depth"]})
        st, tree = h.get_expand(f"namespace={ss['namespace']}&object={ss['object']}&relation={ss['relation']}"
                                f"&max-depth={e['max_depth']}")
        if e["tree"] is None:
            assert got == {} and st == 500
        else:
            assert st == 200 and got == {"tree": tree}
            assert trees_equal_unordered(Tree.from_json(tree), Tree.from_json(e["tree"]))
    assert h.grpc_expand({"subject": {"set": {"namespace": ss["namespace"], "object": "no-such-object",
                                              "relation": "no-such-relation"}}}) == {}
    if reg.mapper.namespaces:
        st, _ = h.get_expand("namespace=no-such-namespace&object=x&relation=y")
        assert st == 404
