"""keto_amd -- MI355X-native batched permission-check engine for Ory Keto's check/expand path.

The hot path is HIP (keto_amd/csrc, built into keto_amd/lib/libketogpu.so, C ABI in
include/ketogpu.h); this package is the host-side mirror of the reference's engine surface.
"""
from .ketoapi import RelationTuple, SubjectSet, Tree, trees_equal_unordered  # noqa: F401
from .mapper import Interner, Mapper, NamespaceNotFound, SUBJECT_ID  # noqa: F401
from .namespace import (ComputedSubjectSet, InvertResult, Namespace, Relation, SubjectSetRewrite,  # noqa: F401
                        TupleToSubjectSet, compile_program, namespace_from_json)


def __getattr__(name):  # engine pieces load the HIP library lazily
    if name in ("Engine", "ExpandEngine", "Snapshot", "Registry", "Config", "CheckError", "Result", "queries_array"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
