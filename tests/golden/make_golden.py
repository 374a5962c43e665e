"""Writes the golden fixtures of the check/expand path as JSON data.

Each fixture is a transcription (as data: inputs + expected outputs) of a known-answer test
that the reference holds for this path; the source file:line is recorded in every case.
Random UUIDs of the reference tests (uuid.NewV4) are replaced by distinct names -- only
identity matters to the engine.  Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=False)
        f.write("\n")


# --------------------------------------------------------------------------- check engine
# internal/check/engine_test.go
engine_cases = [
    {"name": "respects max depth", "source": "internal/check/engine_test.go:72-116",
     "namespaces": [{"name": "test"}],
     "tuples": ["test:object#admin@user", "test:object#owner@test:object#admin",
                "test:object#access@test:object#owner"],
     "checks": [
         {"tuple": "test:object#access@user", "max_depth": 2, "global_max_depth": 5, "allowed": False},
         {"tuple": "test:object#access@user", "max_depth": 3, "global_max_depth": 5, "allowed": True},
         {"tuple": "test:object#access@user", "max_depth": 3, "global_max_depth": 2, "allowed": False},
         {"tuple": "test:object#access@user", "max_depth": 0, "global_max_depth": 3, "allowed": True}]},
    {"name": "direct inclusion", "source": "internal/check/engine_test.go:118-134",
     "namespaces": [{"name": "direct inclusion"}],
     "tuples": ["direct inclusion:obj-1#access@user-1"],
     "checks": [{"tuple": "direct inclusion:obj-1#access@user-1", "max_depth": 0, "global_max_depth": 5,
                 "allowed": True}]},
    {"name": "indirect inclusion level 1", "source": "internal/check/engine_test.go:136-173",
     "namespaces": [{"name": "sofa"}],
     "tuples": ["sofa:dust#have to remove@(sofa:dust#producer)", "sofa:dust#producer@mark"],
     "checks": [{"tuple": "sofa:dust#have to remove@mark", "max_depth": 0, "global_max_depth": 5,
                 "allowed": True}]},
    {"name": "direct exclusion", "source": "internal/check/engine_test.go:175-197",
     "namespaces": [{"name": "direct exclusion"}],
     "tuples": ["direct exclusion:obj-1#relation@user-1"],
     "checks": [{"tuple": "direct exclusion:obj-1#relation@user-2", "max_depth": 0, "global_max_depth": 5,
                 "allowed": False}]},
    {"name": "wrong object ID", "source": "internal/check/engine_test.go:199-227",
     "namespaces": [{"name": ""}],
     "tuples": [":object#access@(:object#owner)", ":other-object#owner@user-1"],
     "checks": [{"tuple": ":object#access@user-1", "max_depth": 0, "global_max_depth": 5, "allowed": False}]},
    {"name": "wrong relation name", "source": "internal/check/engine_test.go:229-265",
     "namespaces": [{"name": "diaries"}],
     "tuples": ["diaries:entry#read@(diaries:entry#author)", "diaries:entry#not author@user-1"],
     "checks": [{"tuple": "diaries:entry#read@user-1", "max_depth": 0, "global_max_depth": 5, "allowed": False}]},
    {"name": "indirect inclusion level 2", "source": "internal/check/engine_test.go:267-331",
     "namespaces": [{"name": "some_namespaces"}, {"name": "organizations"}],
     "tuples": ["some_namespaces:object#write@(some_namespaces:object#owner)",
                "some_namespaces:object#owner@(organizations:org#member)",
                "organizations:org#member@user-1"],
     "checks": [
         {"tuple": "some_namespaces:object#write@user-1", "max_depth": 0, "global_max_depth": 5, "allowed": True},
         {"tuple": "organizations:org#member@user-1", "max_depth": 0, "global_max_depth": 5, "allowed": True}]},
    {"name": "rejects transitive relation", "source": "internal/check/engine_test.go:333-371",
     "namespaces": [{"name": "2"}],
     "tuples": [":file#parent@(:directory#)", ":directory#access@user-1"],
     "checks": [{"tuple": ":file#access@user-1", "max_depth": 0, "global_max_depth": 5, "allowed": False}]},
    {"name": "subject id next to subject set", "source": "internal/check/engine_test.go:373-424",
     "namespaces": [{"name": "39231"}],
     "tuples": ["39231:obj#owner@direct-owner", "39231:obj#owner@(39231:org#member)",
                "39231:org#member@indirect-owner"],
     "checks": [
         {"tuple": "39231:obj#owner@direct-owner", "max_depth": 0, "global_max_depth": 5, "allowed": True},
         {"tuple": "39231:obj#owner@indirect-owner", "max_depth": 0, "global_max_depth": 5, "allowed": True}]},
    {"name": "wide tuple graph", "source": "internal/check/engine_test.go:426-466",
     "namespaces": [{"name": "9234"}],
     "tuples": ["9234:obj#access@(9234:org-0#member)", "9234:obj#access@(9234:org-1#member)",
                "9234:org-0#member@user-0", "9234:org-1#member@user-1",
                "9234:org-0#member@user-2", "9234:org-1#member@user-3"],
     "checks": [{"tuple": f"9234:obj#access@user-{i}", "max_depth": 0, "global_max_depth": 5, "allowed": True}
                for i in range(4)]},
    {"name": "circular tuples", "source": "internal/check/engine_test.go:468-519",
     "namespaces": [{"name": "7743"}],
     "tuples": ["7743:Sendlinger Tor#connected@(7743:Odeonsplatz#connected)",
                "7743:Odeonsplatz#connected@(7743:Central Station#connected)",
                "7743:Central Station#connected@(7743:Sendlinger Tor#connected)"],
     "checks": [{"tuple": "7743:Sendlinger Tor#connected@Central Station", "max_depth": 0,
                 "global_max_depth": 5, "allowed": False}]},
]

# --------------------------------------------------------------------------- rewrites
# internal/check/rewrites_test.go:20-86 (namespaces), :105-128 (tuples), :130-215 (cases, depth 100)
rewrite_namespaces = [
    {"name": "doc", "relations": [
        {"name": "owner"},
        {"name": "editor", "rewrite": {"operator": "or", "children": [{"relation": "owner"}]}},
        {"name": "viewer", "rewrite": {"operator": "or", "children": [
            {"relation": "editor"},
            {"relation": "parent", "computed_subject_set_relation": "viewer"}]}}]},
    {"name": "group", "relations": [{"name": "member"}]},
    {"name": "level", "relations": [{"name": "member"}]},
    {"name": "resource", "relations": [
        {"name": "level"},
        {"name": "viewer", "rewrite": {"operator": "or", "children": [
            {"relation": "owner", "computed_subject_set_relation": "member"}]}},
        {"name": "owner", "rewrite": {"operator": "or", "children": [
            {"relation": "owner", "computed_subject_set_relation": "member"}]}},
        {"name": "read", "rewrite": {"operator": "or", "children": [
            {"relation": "viewer"}, {"relation": "owner"}]}},
        {"name": "update", "rewrite": {"operator": "or", "children": [{"relation": "owner"}]}},
        {"name": "delete", "rewrite": {"operator": "and", "children": [
            {"relation": "owner"},
            {"relation": "level", "computed_subject_set_relation": "member"}]}}]},
    {"name": "acl", "relations": [
        {"name": "allow"}, {"name": "deny"},
        {"name": "access", "rewrite": {"operator": "and", "children": [
            {"relation": "allow"}, {"inverted": {"relation": "deny"}}]}}]},
]
rewrite_tuples = [
    "doc:document#owner@user", "doc:doc_in_folder#parent@doc:folder#...", "doc:folder#owner@user",
    "doc:file#parent@doc:folder_c#...", "doc:folder_c#parent@doc:folder_b#...",
    "doc:folder_b#parent@doc:folder_a#...", "doc:folder_a#owner@user",
    "group:editors#member@mark", "level:superadmin#member@mark", "level:superadmin#member@sandy",
    "resource:topsecret#owner@group:editors#...", "resource:topsecret#level@level:superadmin#...",
    "resource:topsecret#owner@mike",
    "acl:document#allow@alice", "acl:document#allow@bob", "acl:document#allow@mallory",
    "acl:document#deny@mallory",
]
rewrite_expect = [
    ("doc:document#owner@user", True), ("doc:document#editor@user", True), ("doc:document#viewer@user", True),
    ("doc:document#editor@nobody", False), ("doc:folder#viewer@user", True),
    ("doc:doc_in_folder#viewer@user", True), ("doc:doc_in_folder#viewer@nobody", False),
    ("doc:another_doc#viewer@user", False), ("doc:file#viewer@user", True),
    ("level:superadmin#member@mark", True), ("resource:topsecret#owner@mark", True),
    ("resource:topsecret#delete@mark", True), ("resource:topsecret#update@mike", True),
    ("level:superadmin#member@mike", False), ("resource:topsecret#delete@mike", False),
    ("resource:topsecret#delete@sandy", False), ("acl:document#access@alice", True),
    ("acl:document#access@bob", True), ("acl:document#allow@mallory", True),
    ("acl:document#access@mallory", False),
]
# expectedPaths (rewrites_test.go:183-187, :202): labels from the check tree's root down one branch
# each ("*" = any label; the "and" root has no tuple), asserted with hasPath (:263-288)
rewrite_paths = {
    "resource:topsecret#delete@mark": [
        ["*", "resource:topsecret#delete@mark", "level:superadmin#member@mark"],
        ["*", "resource:topsecret#delete@mark", "resource:topsecret#owner@mark", "group:editors#member@mark"]],
    "acl:document#access@alice": [["*", "acl:document#access@alice", "acl:document#allow@alice"]],
}
rewrite_cases = [{
    "name": "usersets rewrites", "source": "internal/check/rewrites_test.go:101-257",
    "namespaces": rewrite_namespaces, "tuples": rewrite_tuples,
    "checks": [dict({"tuple": q, "max_depth": 100, "global_max_depth": 5, "allowed": a},
                    **({"paths": rewrite_paths[q]} if q in rewrite_paths else {})) for q, a in rewrite_expect]}]

# --------------------------------------------------------------------------- expand
# internal/expand/engine_test.go
def leaf_id(s):
    return {"type": "leaf", "tuple": {"namespace": "", "object": "", "relation": "", "subject_id": s}}


def sset(ns, obj, rel):
    return {"namespace": ns, "object": obj, "relation": rel}


def node(t, ss, children=None):
    d = {"type": t, "tuple": {"namespace": "", "object": "", "relation": "", "subject_set": ss}}
    if children:
        d["children"] = children
    return d


expand_cases = [
    {"name": "returns SubjectID on expand", "source": "internal/expand/engine_test.go:50-60",
     "namespaces": [], "tuples": [],
     "expands": [{"subject_id": "user", "max_depth": 100, "global_max_depth": 5, "tree": leaf_id("user")}]},
    {"name": "expands one level", "source": "internal/expand/engine_test.go:62-102",
     "namespaces": [{"name": ""}], "tuples": [":boulder-group#member@tommy", ":boulder-group#member@paul"],
     "expands": [{"subject_set": sset("", "boulder-group", "member"), "max_depth": 100, "global_max_depth": 5,
                  "tree": node("union", sset("", "boulder-group", "member"), [leaf_id("paul"), leaf_id("tommy")])}]},
    {"name": "expands two levels", "source": "internal/expand/engine_test.go:104-181",
     "namespaces": [{"name": ""}],
     "tuples": [":root#transitive member@(:g1#member)", ":g1#member@u1", ":g1#member@u2", ":g1#member@u3",
                ":root#transitive member@(:g2#member)", ":g2#member@u4", ":g2#member@u5", ":g2#member@u6"],
     "expands": [{"subject_set": sset("", "root", "transitive member"), "max_depth": 100, "global_max_depth": 5,
                  "tree": node("union", sset("", "root", "transitive member"), [
                      node("union", sset("", "g1", "member"), [leaf_id("u1"), leaf_id("u2"), leaf_id("u3")]),
                      node("union", sset("", "g2", "member"), [leaf_id("u4"), leaf_id("u5"), leaf_id("u6")])])}]},
    {"name": "respects max depth", "source": "internal/expand/engine_test.go:183-237",
     "namespaces": [{"name": ""}],
     "tuples": [":id0#child@(:id1#child)", ":id1#child@(:id2#child)", ":id2#child@(:id3#child)",
                ":id3#child@(:id4#child)"],
     "expands": [{"subject_set": sset("", "id0", "child"), "max_depth": 4, "global_max_depth": 5, "ordered": True,
                  "tree": node("union", sset("", "id0", "child"), [
                      node("union", sset("", "id1", "child"), [
                          node("union", sset("", "id2", "child"), [
                              node("leaf", sset("", "id3", "child"))])])])}]},
    {"name": "paginates", "source": "internal/expand/engine_test.go:239-269",
     "namespaces": [{"name": ""}],
     "tuples": [":root#access@user-0", ":root#access@user-1", ":root#access@user-2", ":root#access@user-3"],
     "expands": [{"subject_set": sset("", "root", "access"), "max_depth": 10, "global_max_depth": 5,
                  "tree": node("union", sset("", "root", "access"), [leaf_id(f"user-{i}") for i in range(4)])}]},
    {"name": "handles subject sets as leaf", "source": "internal/expand/engine_test.go:271-300",
     "namespaces": [{"name": ""}], "tuples": [":a#rel@(:b#sr)"],
     "expands": [{"subject_set": sset("", "a", "rel"), "max_depth": 100, "global_max_depth": 5, "ordered": True,
                  "tree": node("union", sset("", "a", "rel"), [node("leaf", sset("", "b", "sr"))])}]},
    {"name": "circular tuples", "source": "internal/expand/engine_test.go:302-373",
     "namespaces": [{"name": "92384"}],
     "tuples": ["92384:Sendlinger Tor#connected@(92384:Odeonsplatz#connected)",
                "92384:Odeonsplatz#connected@(92384:Central Station#connected)",
                "92384:Central Station#connected@(92384:Sendlinger Tor#connected)"],
     "expands": [{"subject_set": sset("92384", "Sendlinger Tor", "connected"), "max_depth": 100,
                  "global_max_depth": 5, "ordered": True,
                  "tree": node("union", sset("92384", "Sendlinger Tor", "connected"), [
                      node("union", sset("92384", "Odeonsplatz", "connected"), [
                          node("union", sset("92384", "Central Station", "connected"), [
                              node("leaf", sset("92384", "Sendlinger Tor", "connected"))])])])}]},
    {"name": "expand handler returns tree", "source": "internal/expand/handler_test.go:64-119",
     "namespaces": [{"name": "expand handler"}],
     "tuples": ["expand handler:root#parent of@child0", "expand handler:root#parent of@child1"],
     "expands": [{"subject_set": sset("expand handler", "root", "parent of"), "max_depth": 2, "global_max_depth": 5,
                  "tree": node("union", sset("expand handler", "root", "parent of"),
                               [leaf_id("child0"), leaf_id("child1")])}]},
    {"name": "unknown subject set expands to nil", "source": "internal/expand/engine.go:70-71",
     "namespaces": [{"name": ""}], "tuples": [":a#rel@x"],
     "expands": [{"subject_set": sset("", "nope", "rel"), "max_depth": 3, "global_max_depth": 5, "tree": None}]},
]

# --------------------------------------------------------------------------- cat videos (C1)
# contrib/cat-videos-example/relation-tuples/*.json, keto.yml (namespace videos), up.sh:22-23
cat_dir = "contrib/cat-videos-example/relation-tuples"
cat_cases = [{
    "name": "cat videos", "source": "contrib/cat-videos-example (relation-tuples/*.json, up.sh:22-23)",
    "namespaces": [{"name": "videos", "id": 0}],
    "tuples": ["videos:/cats/1.mp4#owner@(videos:/cats#owner)",
               "videos:/cats/1.mp4#view@(videos:/cats/1.mp4#owner)",
               "videos:/cats/1.mp4#view@*",
               "videos:/cats/2.mp4#owner@(videos:/cats#owner)",
               "videos:/cats/2.mp4#view@(videos:/cats/2.mp4#owner)",
               "videos:/cats#owner@cat lady",
               "videos:/cats#view@(videos:/cats#owner)"],
    "checks": [
        {"tuple": "videos:/cats/1.mp4#view@*", "max_depth": 0, "global_max_depth": 5, "allowed": True},
        {"tuple": "videos:/cats/1.mp4#view@cat lady", "max_depth": 0, "global_max_depth": 5, "allowed": True},
        {"tuple": "videos:/cats/2.mp4#view@*", "max_depth": 0, "global_max_depth": 5, "allowed": False}],
    "expands": [{"subject_set": sset("videos", "/cats/2.mp4", "view"), "max_depth": 0, "global_max_depth": 5,
                 "tree": node("union", sset("videos", "/cats/2.mp4", "view"), [
                     node("union", sset("videos", "/cats/2.mp4", "owner"), [
                         node("union", sset("videos", "/cats", "owner"), [leaf_id("cat lady")])])])}]}]

# --------------------------------------------------------------------------- docs code samples
docs_root = "/root/reference/contrib/docs-code-samples"
beach_expected = None
p = os.path.join(docs_root, "expand-api-display-access/01-expand-beach/expected_output.json")
if os.path.exists(p):
    with open(p) as f:
        beach_expected = json.load(f)
else:  # keep the committed copy when the reference is absent
    with open(os.path.join(HERE, "docs_samples.json")) as f:
        beach_expected = json.load(f)[0]["expands"][0]["tree"]
docs_cases = [
    {"name": "expand api display access", "source":
        "contrib/docs-code-samples/expand-api-display-access (00-create-tuples/cli.sh, 01-expand-beach)",
     "namespaces": [{"name": "files", "id": 1}, {"name": "directories", "id": 2}],
     "tuples": ["directories:/photos#owner@maureen", "files:/photos/beach.jpg#owner@maureen",
                "files:/photos/mountains.jpg#owner@laura", "directories:/photos#access@laura",
                "directories:/photos#access@(directories:/photos#owner)",
                "files:/photos/beach.jpg#access@(files:/photos/beach.jpg#owner)",
                "files:/photos/beach.jpg#access@(directories:/photos#access)",
                "files:/photos/mountains.jpg#access@(files:/photos/mountains.jpg#owner)",
                "files:/photos/mountains.jpg#access@(directories:/photos#access)"],
     "expands": [{"subject_set": sset("files", "/photos/beach.jpg", "access"), "max_depth": 3,
                  "global_max_depth": 5, "tree": beach_expected}]},
    {"name": "simple access check", "source": "contrib/docs-code-samples/simple-access-check-guide",
     "namespaces": [{"name": "messages", "id": 1}],
     "tuples": ["messages:02y_15_4w350m3#decypher@john"],
     "checks": [{"tuple": "messages:02y_15_4w350m3#decypher@john", "max_depth": 0, "global_max_depth": 5,
                 "allowed": True}]},
]

if __name__ == "__main__":
    dump("engine_test.json", engine_cases)
    dump("rewrites_test.json", rewrite_cases)
    dump("expand_test.json", expand_cases)
    dump("cat_videos.json", cat_cases)
    dump("docs_samples.json", docs_cases)
    print("wrote golden fixtures to", HERE)
