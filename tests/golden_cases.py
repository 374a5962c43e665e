"""Helpers that load tests/golden/*.json into interned ids (test utility, not product)."""
import json
import os

from keto_amd.ketoapi import RelationTuple, SubjectSet, Tree
from keto_amd.mapper import Interner, SUBJECT_ID
from keto_amd.namespace import compile_program, namespace_from_json

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def all_cases(kind):
    out = []
    for fn in ("engine_test.json", "rewrites_test.json", "expand_test.json", "cat_videos.json", "docs_samples.json"):
        for c in load(fn):
            if c.get(kind):
                out.append((fn, c))
    return out


class Case:
    def __init__(self, case):
        self.case = case
        self.it = Interner()
        self.namespaces = [namespace_from_json(n) for n in case["namespaces"]]
        self.prog = compile_program(self.namespaces, self.it, lower_ttu=False)  # the oracle: as written
        self.tuples = [RelationTuple.from_string(s) for s in case["tuples"]]
        self.arr = self.it.tuples_array(self.tuples)

    def query(self, s):
        return self.it.tuple_ids(RelationTuple.from_string(s))

    def expand_root(self, e):
        if e.get("subject_id") is not None:
            return SUBJECT_ID, self.it.obj_id(e["subject_id"]), 0
        ss = e["subject_set"]
        return self.it.subject_set_ids(SubjectSet(ss["namespace"], ss["object"], ss["relation"]))

    @staticmethod
    def expected_tree(e):
        return None if e["tree"] is None else Tree.from_json(e["tree"])
