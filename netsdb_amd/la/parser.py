"""LA DSL lexer + recursive-descent parser (reference grammar: src/linearAlgebraDSL/source/LAParser.y,
tokens: LALexer.l).  Produces a list of (identifier, AST) statements; AST nodes are tuples:

    ("id", name) | ("num", value) | ("init", kind, args) | ("bin", op, lhs, rhs)
    ("post", op, expr) | ("func", name, expr) | ("dup", name, expr, size, num)
"""
from __future__ import annotations

import re
from typing import List, Tuple


class LAParseError(ValueError):
    pass


_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+) |
    (?P<comment>\#[^\n]*|//[^\n]*) |
    (?P<str>"(?:[^"\\]|\\.)*") |
    (?P<op>%\*%|'\*|\^-1|\^T|[=+\-*(),]) |
    (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\d+[eE][-+]?\d+|\.\d+|\d+) |
    (?P<id>[A-Za-z_][A-Za-z0-9_]*)
""", re.VERBOSE)

_INIT = {"zeros", "ones", "identity", "load"}
_FUNCS = {"max", "min", "rowMax", "rowMin", "rowSum", "colMax", "colMin", "colSum"}
_DUP = {"duplicateRow", "duplicateCol"}


def tokenize(src: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    while pos < len(src):
        m = _TOKEN_RE.match(src, pos)
        if not m:
            raise LAParseError(f"unexpected character {src[pos]!r} at offset {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind in ("ws", "comment"):
            continue
        out.append((kind, m.group()))
    out.append(("eof", ""))
    return out


class _P:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self):
        return self.t[self.i]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, kind, val=None):
        k, v = self.next()
        if k != kind or (val is not None and v != val):
            raise LAParseError(f"expected {val or kind}, got {v!r}")
        return v

    def statements(self):
        out = []
        while self.peek()[0] != "eof":
            name = self.expect("id")
            self.expect("op", "=")
            out.append((name, self.expression()))
        return out

    def expression(self):
        node = self.multiplicative()
        while self.peek() in (("op", "+"), ("op", "-")):
            op = self.next()[1]
            node = ("bin", op, node, self.multiplicative())
        return node

    def multiplicative(self):
        node = self.postfix()
        while self.peek() in (("op", "%*%"), ("op", "*"), ("op", "'*")):
            op = self.next()[1]
            node = ("bin", op, node, self.postfix())
        return node

    def postfix(self):
        node = self.primary()
        while self.peek() in (("op", "^T"), ("op", "^-1")):
            node = ("post", self.next()[1], node)
        return node

    def _int(self):
        return int(self.expect("num"))

    def primary(self):
        k, v = self.peek()
        if k == "num":
            self.next()
            return ("num", float(v))
        if k == "op" and v == "(":
            self.next()
            e = self.expression()
            self.expect("op", ")")
            return e
        if k == "id":
            self.next()
            if v in _INIT:
                self.expect("op", "(")
                if v == "identity":
                    args = [self._int()]
                    self.expect("op", ",")
                    args.append(self._int())
                else:
                    args = [self._int()]
                    for _ in range(3):
                        self.expect("op", ",")
                        args.append(self._int())
                    if v == "load":
                        self.expect("op", ",")
                        args.append(self.expect("str")[1:-1])
                self.expect("op", ")")
                return ("init", v, args)
            if v in _FUNCS:
                self.expect("op", "(")
                e = self.expression()
                self.expect("op", ")")
                return ("func", v, e)
            if v in _DUP:
                self.expect("op", "(")
                e = self.expression()
                self.expect("op", ",")
                a = self._int()
                self.expect("op", ",")
                b = self._int()
                self.expect("op", ")")
                return ("dup", v, e, a, b)
            return ("id", v)
        raise LAParseError(f"unexpected token {v!r}")


def parse(src: str):
    return _P(tokenize(src)).statements()


__all__ = ["parse", "tokenize", "LAParseError"]
