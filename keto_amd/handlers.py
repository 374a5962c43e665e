"""Request handling of the check and expand APIs above the engines (the transport itself -- HTTP
routing, gRPC servers -- is out of scope): request decoding, the unknown-namespace
rule, status mirroring and the response shapes, as the reference's handlers do them.

  REST  GET/POST /relation-tuples/check            200 {"allowed": true} | 403 {"allowed": false}
        GET/POST /relation-tuples/check/openapi    200 {"allowed": ...} always
                                                    internal/check/handler.go:101-232
        GET /relation-tuples/expand                 internal/expand/handler.go:81-107
  gRPC  CheckService.Check                          internal/check/handler.go:234-275
        ExpandService.Expand                        internal/expand/handler.go:109-146

An unknown namespace is "not allowed" over REST (handler.go:156-160, 221-225) but an error over gRPC
(:261-264, the mapper's herodot.ErrNotFound).  Request errors are herodot's 400s
(ketoapi/public_api_definitions.go:15-19, x/max_depth.go:10-21); engine errors are 500s.
"""
from __future__ import annotations

import json
import re
from typing import Mapping, Optional, Tuple, Union
from urllib.parse import parse_qs

from .engine import CheckError, Engine, ExpandEngine
from .ketoapi import RelationTuple, SubjectSet, TREE_LEAF
from .mapper import Mapper, NamespaceNotFound

SUBJECT_ID_KEY = "subject_id"
SUBJECT_SET_NS_KEY, SUBJECT_SET_OBJ_KEY, SUBJECT_SET_REL_KEY = ("subject_set.namespace", "subject_set.object",
                                                                "subject_set.relation")


class HandlerError(Exception):
    """A herodot error: HTTP status + message (gRPC code alongside)."""

    GRPC = {400: 3, 404: 5, 500: 13}  # InvalidArgument, NotFound, Internal

    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status
        self.message = message

    @property
    def grpc_code(self) -> int:
        return self.GRPC.get(self.status, 2)

    def body(self) -> dict:
        return {"error": {"code": self.status, "message": self.message}}


def _bad(msg: str) -> HandlerError:
    return HandlerError(400, msg)


ERR_DROPPED_SUBJECT_KEY = 'provide "subject_id" or "subject_set.*"; support for "subject" was dropped'
ERR_DUPLICATE_SUBJECT = "exactly one of subject_set or subject_id has to be provided"
ERR_INCOMPLETE_SUBJECT = 'incomplete subject, provide "subject_id" or a complete "subject_set.*"'
ERR_NIL_SUBJECT = "subject is not allowed to be nil"
ERR_INCOMPLETE_TUPLE = 'incomplete tuple, provide "namespace", "object", "relation", and a subject'

Query = Mapping[str, Union[str, list]]


def parse_query(q: Union[str, Query]) -> dict:
    """url.Values: a raw query string or a mapping; values keep every occurrence (Get = the first)."""
    if isinstance(q, str):
        return parse_qs(q.lstrip("?"), keep_blank_values=True)
    return {k: (v if isinstance(v, list) else [v]) for k, v in q.items()}


def _get(q: dict, k: str) -> str:
    v = q.get(k)
    return v[0] if v else ""


_GO_INT = re.compile(r"^[+-]?(0[xX][0-9a-fA-F_]+|0[bB][01_]+|0[oO][0-7_]+|0[0-7_]*|[1-9][0-9_]*)$")


def parse_go_int(s: str) -> int:
    """strconv.ParseInt(s, 0, 0): sign, base prefix 0x / 0b / 0o or a leading 0 (octal), underscores
    only between digits after a prefix; 64-bit range."""
    if not _GO_INT.match(s) or "__" in s or s.endswith("_"):
        raise ValueError(s)
    neg = s.startswith("-")
    body = s.lstrip("+-")
    if "_" in body and not (len(body) > 1 and body[0] == "0"):
        raise ValueError(s)  # underscores need a base prefix
    body = body.replace("_", "")
    if len(body) > 1 and body[0] == "0" and body[1] not in "xXbBoO":
        v = int(body[1:], 8)
    else:
        v = int(body, 0)
    v = -v if neg else v
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError(s)
    return v


def max_depth_from_query(q: dict) -> int:
    """x.GetMaxDepthFromQuery (internal/x/max_depth.go:10-21): absent -> 0 (the global default)."""
    if "max-depth" not in q:
        return 0
    s = _get(q, "max-depth")
    try:
        return parse_go_int(s)
    except ValueError:
        raise _bad(f"unable to parse 'max-depth' query parameter to int: {s!r}")


def tuple_from_url_query(q: dict) -> RelationTuple:
    """RelationTuple.FromURLQuery (ketoapi/enc_url_query.go:12-97)."""
    if "subject" in q:
        raise _bad(ERR_DROPPED_SUBJECT_KEY)
    has_id = SUBJECT_ID_KEY in q
    has_set = [k in q for k in (SUBJECT_SET_NS_KEY, SUBJECT_SET_OBJ_KEY, SUBJECT_SET_REL_KEY)]
    sid: Optional[str] = None
    sset: Optional[SubjectSet] = None
    if not has_id and not any(has_set):
        pass
    elif has_id and any(has_set):
        raise _bad(ERR_DUPLICATE_SUBJECT)
    elif has_id:
        sid = _get(q, SUBJECT_ID_KEY)
    elif all(has_set):
        sset = SubjectSet(_get(q, SUBJECT_SET_NS_KEY), _get(q, SUBJECT_SET_OBJ_KEY), _get(q, SUBJECT_SET_REL_KEY))
    else:
        raise _bad(ERR_INCOMPLETE_SUBJECT)
    if sid is None and sset is None:
        raise _bad(ERR_NIL_SUBJECT)
    if "namespace" not in q or "object" not in q or "relation" not in q:
        raise _bad(ERR_INCOMPLETE_TUPLE)
    return RelationTuple(_get(q, "namespace"), _get(q, "object"), _get(q, "relation"), sid, sset)


def tuple_from_json(body: Union[bytes, str, dict]) -> RelationTuple:
    """json.Decode into ketoapi.RelationTuple (handler.go:215-218); absent fields stay empty."""
    try:
        d = json.loads(body) if isinstance(body, (bytes, str)) else body
        if not isinstance(d, dict):
            raise ValueError("expected a JSON object")
        return RelationTuple.from_json(d)
    except (ValueError, AttributeError, TypeError) as e:
        raise _bad(f"could not unmarshal json: {e}")


class CheckHandler:
    """internal/check/handler.go: REST (mirrored / openapi) and gRPC Check over one engine."""

    def __init__(self, engine: Engine, mapper: Mapper):
        self.engine, self.mapper = engine, mapper

    def _check(self, t: RelationTuple, max_depth: int, unknown_ns_false: bool) -> bool:
        if t.subject_id is None and t.subject_set is None:
            raise _bad(ERR_NIL_SUBJECT)
        try:
            self.mapper.from_tuple(t)
        except NamespaceNotFound as e:
            if unknown_ns_false:  # handler.go:156-160 / 221-225: "not allowed", not "not found"
                return False
            raise HandlerError(404, f"Unable to locate the resource: namespace {e.args[0]!r}")
        try:
            return self.engine.check_is_member(t, max_depth)
        except CheckError as e:
            raise HandlerError(500, str(e))

    def _rest(self, produce, mirror_status: bool) -> Tuple[int, dict]:
        try:
            allowed = produce()
        except HandlerError as e:
            return e.status, e.body()
        if allowed or not mirror_status:
            return 200, {"allowed": allowed}
        return 403, {"allowed": False}  # handler.go:138-141

    def get_check(self, query: Union[str, Query], mirror_status: bool = True) -> Tuple[int, dict]:
        """GET /relation-tuples/check (mirror_status) or /relation-tuples/check/openapi."""
        def produce():
            q = parse_query(query)
            d = max_depth_from_query(q)
            return self._check(tuple_from_url_query(q), d, True)
        return self._rest(produce, mirror_status)

    def post_check(self, body: Union[bytes, str, dict], query: Union[str, Query] = "",
                   mirror_status: bool = True) -> Tuple[int, dict]:
        """POST /relation-tuples/check (mirror_status) or /relation-tuples/check/openapi."""
        def produce():
            d = max_depth_from_query(parse_query(query))
            return self._check(tuple_from_json(body), d, True)
        return self._rest(produce, mirror_status)

    def grpc_check(self, req: dict) -> dict:
        """CheckService.Check (handler.go:234-275): req = {"tuple": {...}} or the deprecated flat
        fields, plus "max_depth".  Raises HandlerError (grpc_code) on failure."""
        src = req.get("tuple") if req.get("tuple") is not None else req
        sub = src.get("subject")
        if not sub:
            raise _bad(ERR_NIL_SUBJECT)
        if "id" in sub:
            t = RelationTuple(src.get("namespace", ""), src.get("object", ""), src.get("relation", ""),
                              subject_id=sub["id"])
        else:
            s = sub.get("set") or {}
            t = RelationTuple(src.get("namespace", ""), src.get("object", ""), src.get("relation", ""),
                              subject_set=SubjectSet(s.get("namespace", ""), s.get("object", ""), s.get("relation", "")))
        allowed = self._check(t, int(req.get("max_depth", 0)), False)
        return {"allowed": allowed, "snaptoken": "not yet implemented"}


class ExpandHandler:
    """internal/expand/handler.go: REST GET and gRPC Expand over one expand engine."""

    def __init__(self, engine: ExpandEngine, mapper: Mapper):
        self.engine, self.mapper = engine, mapper

    def _tree(self, s: SubjectSet, max_depth: int):
        try:
            self.mapper.from_subject_set(s)
        except NamespaceNotFound as e:
            raise HandlerError(404, f"Unable to locate the resource: namespace {e.args[0]!r}")
        return self.engine.build_tree(s, max_depth)

    def get_expand(self, query: Union[str, Query]) -> Tuple[int, Optional[dict]]:
        """GET /relation-tuples/expand?namespace=&object=&relation=&max-depth= (handler.go:81-107).
        The reference has no nil guard before Mapper.ToTree (uuid_mapping.go:314 dereferences the
        nil tree of an empty or unknown set): that request fails with a server error here too."""
        try:
            q = parse_query(query)
            d = max_depth_from_query(q)
            s = SubjectSet(_get(q, "namespace"), _get(q, "object"), _get(q, "relation"))
            tree = self._tree(s, d)
        except HandlerError as e:
            return e.status, e.body()
        if tree is None:
            return 500, HandlerError(500, "expand: empty tree (no nil guard in the reference)").body()
        return 200, tree.to_json()

    def grpc_expand(self, req: dict) -> dict:
        """ExpandService.Expand (handler.go:109-146): a subject id is a leaf of itself; a nil tree is
        an empty response (:136-138)."""
        sub = req.get("subject") or {}
        if "id" in sub:
            return {"tree": {"node_type": TREE_LEAF, "subject": {"id": sub["id"]}}}
        s = sub.get("set") or {}
        tree = self._tree(SubjectSet(s.get("namespace", ""), s.get("object", ""), s.get("relation", "")),
                          int(req.get("max_depth", 0)))
        if tree is None:
            return {}
        return {"tree": tree.to_json()}
