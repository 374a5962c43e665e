"""OPL (Ory Permission Language) front end: TypeScript-like namespace classes -> namespace configs.

A restatement of the reference's ``internal/schema`` package (lexer.go, parser.go, typechecks.go,
limits.go); the output is the ``keto_amd.namespace`` AST that ``compile_program`` turns into the
engine's rewrite program.  Behaviour kept from the reference, quirks included:

  * lexer (lexer.go:237-319): multi-rune tokens ``=> || &&`` before one-rune ones, ``//`` and
    ``/* */`` comments, string literals of letters/digits only, identifiers ``[A-Za-z_][A-Za-z0-9_]*``
  * ``peek`` does NOT skip comments, ``next`` does (parser.go:31-50)
  * binary ``&&`` / ``||`` are left-associative with NO precedence: an operator makes the tree so far
    its first child (parser.go:317-324); ``(`` groups and ``!`` nest, at most
    ``expressionNestingMaxDepth`` = 10 deep (limits.go:10, parser.go:281-286,355-361)
  * after a plain expression the parser still expects an expression (parser.go:344-349), so two
    expressions in a row are both children of the current node
  * ``simplifyExpression`` merges a child into its parent when both are the same operator, and only
    recurses into merged children (parser.go:465-483)
  * type checks run after the whole input is parsed and only add errors (typechecks.go:41-127)

``parse(text)`` returns ``(namespaces, errors)`` like ``schema.Parse`` (parser.go:24-29).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

from .namespace import (ComputedSubjectSet, InvertResult, Namespace, OP_AND, OP_OR, Relation, RelationType,
                        SubjectSetRewrite, TupleToSubjectSet, as_rewrite)

EXPRESSION_NESTING_MAX_DEPTH = 10        # limits.go:10
TUPLE_TO_SUBJECT_SET_TYPECHECK_MAX_DEPTH = 10  # limits.go:6

# item types (lexer.go:37-76)
ERROR, EOF, IDENT, COMMENT, STRING = "error", "EOF", "identifier", "comment", "string literal"
KW_CLASS, KW_IMPLEMENTS, KW_THIS, KW_CTX = "class", "implements", "this", "ctx"
AND, OR, NOT, ASSIGN, ARROW, DOT, COLON, COMMA, UNION = "&&", "||", "!", "=", "=>", ".", ":", ",", "|"
PAREN_L, PAREN_R, BRACE_L, BRACE_R, BRACKET_L, BRACKET_R, ANGLE_L, ANGLE_R = "(", ")", "{", "}", "[", "]", "<", ">"

_SPACES = "\t\n\v\f\r "
_DIGITS = "0123456789"
_LETTERS = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ_"
_ONE_RUNE = {":": COLON, ".": DOT, "(": PAREN_L, ")": PAREN_R, "[": BRACKET_L, "]": BRACKET_R, "{": BRACE_L,
             "}": BRACE_R, "<": ANGLE_L, ">": ANGLE_R, "=": ASSIGN, ",": COMMA, "|": UNION, "!": NOT}
_MULTI_RUNE = {"=>": ARROW, "||": OR, "&&": AND}
_KEYWORDS = {"class": KW_CLASS, "implements": KW_IMPLEMENTS, "this": KW_THIS, "ctx": KW_CTX}


@dataclass
class Item:
    typ: str
    val: str
    start: int
    end: int

    def __str__(self) -> str:  # lexer.go:87-100
        if self.typ == ERROR:
            return "error: " + self.val
        if self.typ == EOF:
            return "EOF"
        if self.typ in (IDENT, STRING):
            return "'%.10s...'" % self.val if len(self.val) > 10 else "'%s'" % self.val
        return self.val


class Lexer:
    """lexer.go: a state machine emitting items on demand."""

    def __init__(self, text: str):
        self.input = text
        self.pos = 0
        self.start = 0
        self.items: List[Item] = []
        self.state: Optional[Callable[[], Optional[Callable]]] = self._code

    def _emit(self, typ: str) -> None:
        self.items.append(Item(typ, self.input[self.start:self.pos], self.start, self.pos))
        self.start = self.pos

    def _errorf(self, msg: str):
        self.items.append(Item(ERROR, "at %r: %s" % (self.input[self.pos:], msg), self.start, self.pos))
        return None

    def next_item(self) -> Item:
        while True:
            if self.items:
                return self.items.pop(0)
            if self.state is None:
                return Item(ERROR, "broken state", 0, 0)
            self.state = self.state()

    def _peek(self) -> str:
        return self.input[self.pos] if self.pos < len(self.input) else ""

    def _code(self):
        while self.pos < len(self.input) and self.input[self.pos] in _SPACES:
            self.pos += 1
        self.start = self.pos
        r = self._peek()
        if r == "":
            self._emit(EOF)
            return None
        for tok, typ in _MULTI_RUNE.items():
            if self.input.startswith(tok, self.pos):
                self.pos += len(tok)
                self._emit(typ)
                return self._code
        if self.input.startswith("//", self.pos):
            self.pos += 2
            return self._line_comment
        if self.input.startswith("/*", self.pos):
            self.pos += 2
            return self._block_comment
        if r in _ONE_RUNE:
            self.pos += 1
            self._emit(_ONE_RUNE[r])
            return self._code
        if r in "'\"":
            return self._string
        if r in _LETTERS:
            self.pos += 1
            while self.pos < len(self.input) and self.input[self.pos] in _LETTERS + _DIGITS:
                self.pos += 1
            self._emit(_KEYWORDS.get(self.input[self.start:self.pos], IDENT))
            return self._code
        return self._errorf("unexpected token %s" % r)

    def _line_comment(self):
        while self.pos < len(self.input) and self.input[self.pos] != "\n":
            self.pos += 1
        self._emit(COMMENT)
        return self._code

    def _block_comment(self):
        while True:
            if self.pos >= len(self.input):
                return self._errorf("unclosed comment")
            if self.input.startswith("*/", self.pos):
                self.pos += 2
                self._emit(COMMENT)
                return self._code
            self.pos += 1

    def _string(self):
        quote = self.input[self.pos]
        self.pos += 1
        self.start = self.pos
        while self.pos < len(self.input) and self.input[self.pos] in _DIGITS + _LETTERS:
            self.pos += 1
        if self._peek() != quote:
            return self._errorf("unclosed string literal")
        self._emit(STRING)
        self.pos += 1
        self.start = self.pos
        return self._code


def lex(text: str) -> List[Item]:
    """Every item up to and including EOF or the first error (the lexer tests' view)."""
    lx = Lexer(text)
    out = []
    while True:
        it = lx.next_item()
        out.append(it)
        if it.typ in (EOF, ERROR):
            return out


class ParseError(Exception):
    """parse_errors.go: message with the item's source position."""

    def __init__(self, msg: str, item: Item, text: str):
        self.msg, self.item = msg, item
        line, col = _src_pos(text, item.start)
        super().__init__("error from %d:%d: %s" % (line, col, msg))


def _src_pos(text: str, pos: int) -> Tuple[int, int]:
    line, col = 1, 0
    for c in text:
        col += 1
        pos -= 1
        if pos == 0:
            return line, col
        if c == "\n":
            line += 1
            col = 0
    return 0, 0


class _Optional:
    def __init__(self, *tokens: str):
        self.tokens = tokens


class _Parser:
    def __init__(self, text: str):
        self.text = text
        self.lexer = Lexer(text)
        self.namespaces: List[Namespace] = []
        self.ns: Optional[Namespace] = None
        self.errors: List[ParseError] = []
        self.fatal = False
        self.lookahead: Optional[Item] = None
        self.checks: List[Callable[[], None]] = []

    # ---- token plumbing (parser.go:31-163)
    def next(self) -> Item:
        if self.lookahead is not None:
            it, self.lookahead = self.lookahead, None
            return it
        it = self.lexer.next_item()
        while it.typ == COMMENT:
            it = self.lexer.next_item()
        return it

    def peek(self) -> Item:
        if self.lookahead is None:
            self.lookahead = self.lexer.next_item()  # comments included, as in the reference
        return self.lookahead

    def add_err(self, item: Item, msg: str) -> None:
        self.errors.append(ParseError(msg, item, self.text))

    def add_fatal(self, item: Item, msg: str) -> None:
        self.add_err(item, msg)
        self.fatal = True

    def match(self, *tokens) -> Tuple[bool, list]:
        """Strings must match exactly; IDENT captures an identifier or string literal; ITEM captures
        any item; _Optional(...) matches its tokens iff the first one is next."""
        got: list = []
        if self.fatal:
            return False, got
        for tok in tokens:
            if isinstance(tok, _Optional):
                if self.peek().val == tok.tokens[0]:
                    self.next()
                    for t in tok.tokens[1:]:
                        i = self.next()
                        if i.val != t:
                            self.add_fatal(i, "expected %r, got %r" % (t, i.val))
                            return False, got
            elif tok is _IDENT:
                i = self.next()
                if i.typ not in (IDENT, STRING):
                    self.add_fatal(i, "expected identifier, got %s" % i.typ)
                    return False, got
                got.append(i.val)
            elif tok is _ITEM:
                got.append(self.next())
            else:
                i = self.next()
                if i.val != tok:
                    self.add_fatal(i, "expected %r, got %r" % (tok, i.val))
                    return False, got
        return True, got

    # ---- grammar (parser.go:52-461)
    def parse(self):
        while not self.fatal:
            it = self.next()
            if it.typ == EOF:
                break
            if it.typ == ERROR:
                self.add_fatal(it, "fatal: %s" % it.val)
            elif it.typ == KW_CLASS:
                self.parse_class()
        for check in self.checks:  # typechecks.go:41-45
            check()
        return self.namespaces, self.errors

    def parse_class(self) -> None:
        ok, got = self.match(_IDENT, "implements", "Namespace", "{")
        self.ns = Namespace(got[0] if got else "", [])
        while not self.fatal:
            it = self.next()
            if it.typ == BRACE_R:
                self.namespaces.append(self.ns)
                return
            if it.val == "related":
                self.parse_related()
            elif it.val == "permits":
                self.parse_permits()
            else:
                self.add_fatal(it, "expected 'permits' or 'related', got %r" % it.val)
                return

    def parse_related(self) -> None:
        self.match(":", "{")
        while not self.fatal:
            it = self.next()
            if it.typ == BRACE_R:
                return
            if it.typ != IDENT:
                self.add_fatal(it, "expected identifier or '}', got %r" % it.val)
                return
            name = it.val
            types: List[RelationType] = []
            self.match(":")
            t = self.next()
            if t.typ == IDENT:
                if t.val == "SubjectSet":
                    types.append(self.match_subject_set())
                else:
                    types.append(RelationType(t.val))
                    self.checks.append(self._check_namespace_exists(t))
            elif t.typ == PAREN_L:
                types.extend(self.parse_type_union())
            self.match("[", "]")
            self.ns.relations.append(Relation(name, types))

    def match_subject_set(self) -> RelationType:
        _, got = self.match("<", _ITEM, ",", _ITEM, ">")
        ns_item = got[0] if len(got) > 0 else Item(ERROR, "", 0, 0)
        rel_item = got[1] if len(got) > 1 else Item(ERROR, "", 0, 0)
        self.checks.append(self._check_namespace_has_relation(ns_item, rel_item))
        return RelationType(ns_item.val, rel_item.val)

    def parse_type_union(self) -> List[RelationType]:
        types = []
        while not self.fatal:
            _, got = self.match(_ITEM)
            ident = got[0] if got else Item(ERROR, "", 0, 0)
            if ident.val == "SubjectSet":
                types.append(self.match_subject_set())
            else:
                types.append(RelationType(ident.val))
                self.checks.append(self._check_namespace_exists(ident))
            it = self.next()
            if it.typ == PAREN_R:
                return types
            if it.typ != UNION:
                self.add_fatal(it, "expected '|', got %r" % it.val)
        return types

    def parse_permits(self) -> None:
        self.match("=", "{")
        while not self.fatal:
            it = self.next()
            if it.typ == BRACE_R:
                return
            if it.typ != IDENT:
                self.add_fatal(it, "expected identifier or '}', got %r" % it.val)
                return
            self.match(":", "(", "ctx", _Optional(":", "Context"), ")", _Optional(":", "boolean"), "=>")
            rewrite = simplify_expression(self.parse_permission_expressions(COMMA, EXPRESSION_NESTING_MAX_DEPTH))
            if rewrite is None:
                return
            self.ns.relations.append(Relation(it.val, rewrite=rewrite))

    def parse_permission_expressions(self, final: str, depth: int) -> Optional[SubjectSetRewrite]:
        if depth <= 0:
            self.add_fatal(self.peek(), "expression nested too deeply; maximal nesting depth is %d"
                           % EXPRESSION_NESTING_MAX_DEPTH)
            return None
        root: Optional[SubjectSetRewrite] = None
        expect_expression = True
        while not self.fatal:
            it = self.peek()
            if it.typ == PAREN_L:
                self.next()
                child = self.parse_permission_expressions(PAREN_R, depth - 1)
                if child is None:
                    return None
                root = _add_child(root, child)
                expect_expression = False
            elif it.typ == final:
                self.next()
                return root
            elif it.typ == BRACE_R:  # left for parse_permits to consume
                return root
            elif it.typ in (AND, OR):
                self.next()
                root = SubjectSetRewrite([root], OP_AND if it.typ == AND else OP_OR)
                expect_expression = True
            elif it.typ == NOT:
                self.next()
                child = self.parse_not_expression(depth - 1)
                if child is None:
                    return None
                root = _add_child(root, child)
                expect_expression = False
            else:
                if not expect_expression:
                    self.add_fatal(it, "did not expect another expression")
                    return None
                child = self.parse_permission_expression()
                if child is None:
                    return None
                root = _add_child(root, child)
                expect_expression = True  # sic (parser.go:349)
        return None

    def parse_not_expression(self, depth: int):
        if depth <= 0:
            self.add_fatal(self.peek(), "expression nested too deeply; maximal nesting depth is %d"
                           % EXPRESSION_NESTING_MAX_DEPTH)
            return None
        if self.peek().typ == PAREN_L:
            self.next()
            child = self.parse_permission_expressions(PAREN_R, depth - 1)
        else:
            child = self.parse_permission_expression()
        if child is None:
            return None
        return InvertResult(child)

    def parse_permission_expression(self):
        ok, got = self.match("this", ".", "related", ".", _ITEM, ".")
        if not ok:
            return None
        name = got[0]
        it = self.next()
        if it.val == "traverse":
            return self.parse_tuple_to_subject_set(name)
        if it.val == "includes":
            return self.parse_computed_subject_set(name)
        self.add_fatal(it, "expected 'traverse' or 'includes', got %r" % it.val)
        return None

    def parse_tuple_to_subject_set(self, relation: Item):
        ok, _ = self.match("(")
        if not ok:
            return None
        if not self.fatal and self.peek().typ == PAREN_L:
            ok, got = self.match("(", _ITEM, ")")
        else:
            ok, got = self.match(_ITEM)
        if not ok:
            return None
        arg = got[0]
        _, got = self.match("=>", arg.val, ".", _ITEM)
        verb = got[0] if got else Item(ERROR, "", 0, 0)
        if verb.val == "related":
            _, got = self.match(".", _IDENT, ".", "includes", "(", "ctx", ".", "subject", _Optional(","), ")",
                                _Optional(","), ")")
        elif verb.val == "permits":
            _, got = self.match(".", _IDENT, "(", "ctx", ")", ")")
        else:
            self.add_fatal(verb, "expected 'related' or 'permits', got %r" % verb.val)
            return None
        sub_rel = got[0] if got else ""
        self.checks.append(self._check_all_relation_types_have_relation(self.ns, relation, sub_rel))
        self.checks.append(self._check_current_namespace_has_relation(self.ns, relation))
        return TupleToSubjectSet(relation.val, sub_rel)

    def parse_computed_subject_set(self, relation: Item):
        ok, _ = self.match("(", "ctx", ".", "subject", ")")
        if not ok:
            return None
        self.checks.append(self._check_current_namespace_has_relation(self.ns, relation))
        return ComputedSubjectSet(relation.val)

    # ---- type checks (typechecks.go:51-127); run after parsing, they only add errors
    def _find(self, name: str) -> Optional[Namespace]:
        for n in self.namespaces:
            if n.name == name:
                return n
        return None

    def _find_relation(self, ns: str, rel: str) -> Optional[Relation]:
        n = self._find(ns)
        if n is None:
            return None
        for r in n.relations:
            if r.name == rel:
                return r
        return None

    def _check_namespace_exists(self, item: Item):
        def check():
            if self._find(item.val) is None:
                self.add_err(item, "namespace %r was not declared" % item.val)
        return check

    def _check_namespace_has_relation(self, ns_item: Item, rel_item: Item):
        def check():
            n = self._find(ns_item.val)
            if n is None:
                self.add_err(ns_item, "namespace %r was not declared" % ns_item.val)
            elif self._find_relation(ns_item.val, rel_item.val) is None:
                self.add_err(rel_item, "namespace %r did not declare relation %r" % (ns_item.val, rel_item.val))
        return check

    def _check_current_namespace_has_relation(self, current: Namespace, rel: Item):
        name = current.name

        def check():
            if self._find(name) is None:
                self.add_err(rel, "namespace %r was not declared" % name)
            elif self._find_relation(name, rel.val) is None:
                self.add_err(rel, "namespace %r did not declare relation %r" % (name, rel.val))
        return check

    def _check_all_relation_types_have_relation(self, current: Namespace, rtype: Item, relation: str):
        name = current.name

        def rec(ns: str, rtype_val: str, depth: int):
            if depth < 0:
                self.add_err(rtype, "could not typecheck deeply nested SubjectSet further")
                return
            r = self._find_relation(ns, rtype_val)
            if r is None:
                self.add_err(rtype, "relation %r was not declared in namespace %r" % (rtype_val, ns))
                return
            for t in r.types:
                if t.relation == "":
                    if self._find_relation(t.namespace, relation) is None:
                        self.add_err(rtype, "relation %r was not declared in namespace %r" % (relation, t.namespace))
                else:
                    rec(t.namespace, t.relation, depth - 1)

        return lambda: rec(name, rtype.val, TUPLE_TO_SUBJECT_SET_TYPECHECK_MAX_DEPTH)


_IDENT = object()  # match(): an identifier or string literal, captured as its text
_ITEM = object()   # match(): any item, captured


def _add_child(root: Optional[SubjectSetRewrite], child) -> SubjectSetRewrite:
    """parser.go:376-383."""
    if root is None:
        return as_rewrite(child)
    root.children.append(child)
    return root


def simplify_expression(root: Optional[SubjectSetRewrite]) -> Optional[SubjectSetRewrite]:
    """parser.go:465-483: n-ary merge of same-operator children; recursion only into merged ones."""
    if root is None:
        return None
    new_children = []
    for child in root.children:
        if isinstance(child, SubjectSetRewrite) and child.operation == root.operation:
            simplify_expression(child)
            new_children.extend(child.children)
        else:
            new_children.append(child)
    root.children = new_children
    return root


def parse(text: str) -> Tuple[List[Namespace], List[ParseError]]:
    """schema.Parse (internal/schema/parser.go:24-29)."""
    return _Parser(text).parse()


def parse_strict(text: str) -> List[Namespace]:
    """parse() that raises the first error (a config loader's view)."""
    nss, errs = parse(text)
    if errs:
        raise errs[0]
    return nss
