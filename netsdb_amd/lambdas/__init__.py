"""UDF lambda trees (reference: src/lambdas/headers/Lambda.h, LambdaCreationFunctions.h,
AttAccessLambda.h, MethodCallLambda.h, CPlusPlusLambda.h, EqualsLambda.h, AndLambda.h,
SelfLambda.h, DereferenceLambda.h).

A computation's ``get_selection``/``get_projection``/``get_key_projection`` builds a tree from
placeholders (:class:`Arg`, the analogue of ``Handle<T> in1``).  The tree is (a) compiled into
TCAP APPLY/FILTER/HASH atoms, one per node, and (b) evaluated column-at-a-time by the executor:
attribute and method accesses read whole columns (GPU tensors), comparisons/arithmetic are
vectorised, and opaque native lambdas either take columns (``vectorized=True``) or fall back to
object-at-a-time over :class:`RecordView` s.
"""
from __future__ import annotations

import itertools
from typing import Any, Callable, List, Optional, Sequence

import torch

from ..objects.record import RecordBatch, RecordView, column_item
from ..objects.strings import StringColumn


class Arg:
    """Placeholder for the i-th input of a computation (a ``Handle<T>`` parameter)."""

    def __init__(self, index: int, type_: Optional[type] = None):
        self.index = index
        self.type = type_

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        # in1.field -> attribute access (sugar; the reference uses makeLambdaFromMember)
        return AttAccess(self, name)

    def __repr__(self):
        return f"in{self.index}"


class Lambda:
    """Node of a lambda tree."""

    kind = "lambda"

    def __init__(self, children: Sequence["Lambda"] = (), inputs: Sequence[int] = ()):
        self.children = list(children)
        self._inputs = list(inputs)
        self.name: Optional[str] = None

    # -- structure
    def input_indices(self) -> List[int]:
        s = set(self._inputs)
        for c in self.children:
            s.update(c.input_indices())
        return sorted(s)

    def nodes_postorder(self) -> List["Lambda"]:
        out: List[Lambda] = []
        self._postorder(out)
        return out

    def _postorder(self, out: List["Lambda"]) -> None:
        for c in self.children:
            c._postorder(out)
        out.append(self)

    def assign_names(self, counter=None) -> "Lambda":
        counter = counter if counter is not None else itertools.count()
        for n in self.nodes_postorder():
            if n.name is None:
                n.name = f"{n.kind}_{next(counter)}"
        return self

    # -- evaluation: `inputs` are row-aligned RecordBatches (index = computation input index)
    def eval(self, inputs: Sequence[RecordBatch]):
        vals = [c.eval(inputs) for c in self.children]
        return self.eval_node(inputs, vals)

    def eval_node(self, inputs, child_vals):
        raise NotImplementedError

    # -- operators build trees (reference: operator== / operator&& on LambdaTree)
    def __eq__(self, other):  # type: ignore[override]
        return Binary("==", self, _lift(other))

    def __ne__(self, other):  # type: ignore[override]
        return Binary("!=", self, _lift(other))

    def __and__(self, other):
        return Binary("&&", self, _lift(other))

    def __or__(self, other):
        return Binary("||", self, _lift(other))

    def __invert__(self):
        return Unary("!", self)

    def __gt__(self, other):
        return Binary(">", self, _lift(other))

    def __ge__(self, other):
        return Binary(">=", self, _lift(other))

    def __lt__(self, other):
        return Binary("<", self, _lift(other))

    def __le__(self, other):
        return Binary("<=", self, _lift(other))

    def __add__(self, other):
        return Binary("+", self, _lift(other))

    def __sub__(self, other):
        return Binary("-", self, _lift(other))

    def __mul__(self, other):
        return Binary("*", self, _lift(other))

    def __truediv__(self, other):
        return Binary("/", self, _lift(other))

    # literal on the left (``1 - in.l_discount``)
    def __radd__(self, other):
        return Binary("+", _lift(other), self)

    def __rsub__(self, other):
        return Binary("-", _lift(other), self)

    def __rmul__(self, other):
        return Binary("*", _lift(other), self)

    def __rtruediv__(self, other):
        return Binary("/", _lift(other), self)

    def __neg__(self):
        return Binary("-", Literal(0.0), self)

    __hash__ = object.__hash__

    def __repr__(self):
        return f"{self.kind}({', '.join(map(repr, self.children))})"


def _lift(x) -> Lambda:
    if isinstance(x, Lambda):
        return x
    if isinstance(x, Arg):
        return SelfLambda(x)
    return Literal(x)


class Literal(Lambda):
    kind = "literal"

    def __init__(self, value):
        super().__init__()
        self.value = value

    def eval_node(self, inputs, child_vals):
        return self.value


class SelfLambda(Lambda):
    """makeLambdaFromSelf: the input object itself (the whole row of that input)."""

    kind = "self"

    def __init__(self, arg: Arg):
        super().__init__(inputs=[arg.index])
        self.arg = arg

    def eval_node(self, inputs, child_vals):
        return SelfRef(inputs[self.arg.index])


class SelfRef:
    """Column value meaning 'the objects of this batch' (materialised lazily)."""

    __slots__ = ("batch",)

    def __init__(self, batch: RecordBatch):
        self.batch = batch

    def __len__(self):
        return self.batch.n

    def views(self):
        return [RecordView(self.batch, i) for i in range(self.batch.n)]


class AttAccess(Lambda):
    kind = "attAccess"

    def __init__(self, arg: Arg, field: str):
        super().__init__(inputs=[arg.index])
        self.arg = arg
        self.field = field

    def eval_node(self, inputs, child_vals):
        b = inputs[self.arg.index]
        if self.field in b.columns:
            return b.columns[self.field]
        # nested access on an object column is done per record
        return [getattr(v, self.field) for v in SelfRef(b).views()]

    def __repr__(self):
        return f"{self.arg}.{self.field}"


class MethodCall(Lambda):
    kind = "methodCall"

    def __init__(self, arg: Arg, method: str):
        super().__init__(inputs=[arg.index])
        self.arg = arg
        self.method = method

    def eval_node(self, inputs, child_vals):
        b = inputs[self.arg.index]
        t = b.type
        fn = getattr(t, self.method, None) if t is not None else None
        if fn is None:
            raise AttributeError(f"type {t} has no method {self.method}")
        vec = getattr(fn, "__vectorized__", None)
        if vec is not None:
            return vec(b)
        return [fn(v) for v in SelfRef(b).views()]

    def __repr__(self):
        return f"{self.arg}.{self.method}()"


class Native(Lambda):
    """makeLambda(in..., fn): an opaque UDF (CPlusPlusLambda).

    ``vectorized=True``: ``fn`` receives whole columns / batches (SelfRef -> RecordBatch) and must
    return a column of the batch length — this is how tensor UDFs reach the HIP kernels.
    Otherwise ``fn`` is called per record with :class:`RecordView` arguments.
    """

    kind = "native_lambda"

    def __init__(self, args: Sequence[Any], fn: Callable, vectorized: bool = False, tag: Optional[str] = None):
        kids = [_lift(a) for a in args]
        super().__init__(children=kids)
        self.fn = fn
        self.vectorized = vectorized
        self.tag = tag  # optional semantic tag (e.g. 'block_matmul') the planner may pattern-match

    def eval_node(self, inputs, child_vals):
        if self.vectorized:
            args = [v.batch if isinstance(v, SelfRef) else v for v in child_vals]
            return self.fn(*args)
        n = None
        for v in child_vals:
            if isinstance(v, SelfRef):
                n = v.batch.n
                break
            if isinstance(v, RecordBatch):
                n = v.n
                break
            if isinstance(v, (list, StringColumn, torch.Tensor)):
                n = len(v)
                break
        if n is None:
            return self.fn(*child_vals)
        cols = [_row_accessor(v) for v in child_vals]
        return [self.fn(*[c(i) for c in cols]) for i in range(n)]


def _row_accessor(v):
    if isinstance(v, SelfRef):
        b = v.batch
        return lambda i: RecordView(b, i)
    if isinstance(v, RecordBatch):
        return lambda i: RecordView(v, i)
    if isinstance(v, tuple):
        return lambda i: tuple(column_item(c, i) for c in v)
    if isinstance(v, StringColumn):
        lst = v.tolist()                  # one D2H for a row-at-a-time (non-vectorised) lambda
        return lambda i: lst[i]
    if isinstance(v, (list, StringColumn, torch.Tensor)):
        return lambda i: column_item(v, i)
    return lambda i: v


_BIN = {
    "==": lambda a, b: a == b, "!=": lambda a, b: a != b, ">": lambda a, b: a > b, ">=": lambda a, b: a >= b,
    "<": lambda a, b: a < b, "<=": lambda a, b: a <= b, "+": lambda a, b: a + b, "-": lambda a, b: a - b,
    "*": lambda a, b: a * b, "/": lambda a, b: a / b,
}


class Binary(Lambda):
    def __init__(self, op: str, lhs: Lambda, rhs: Lambda):
        super().__init__(children=[lhs, rhs])
        self.op = op
        self.kind = {"==": "==", "&&": "&&", "||": "||"}.get(op, _OPNAME.get(op, op))

    def eval_node(self, inputs, child_vals):
        a, b = child_vals
        if self.op in ("&&", "||"):
            return _logic(self.op, a, b)
        if self.op == "==" or self.op == "!=":
            eq = _equals(a, b)
            return eq if self.op == "==" else _not(eq)
        return _elementwise(_BIN[self.op], a, b)


_OPNAME = {">": "greaterThan", ">=": "greaterEq", "<": "lessThan", "<=": "lessEq", "+": "plus", "-": "minus",
           "*": "times", "/": "divide", "!=": "notEquals"}


class Unary(Lambda):
    kind = "not"

    def __init__(self, op: str, x: Lambda):
        super().__init__(children=[x])
        self.op = op

    def eval_node(self, inputs, child_vals):
        return _not(child_vals[0])


def _to_tensor_col(v):
    if isinstance(v, torch.Tensor):
        return v
    if isinstance(v, list) and v and isinstance(v[0], (bool, int, float)):
        return torch.tensor(v)
    return None


def _equals(a, b):
    if isinstance(a, tuple) and isinstance(b, tuple):
        out = None
        for x, y in zip(a, b):
            e = _equals(x, y)
            out = e if out is None else _logic("&&", out, e)
        return out
    if isinstance(a, str) and isinstance(b, StringColumn):
        a, b = b, a
    if isinstance(a, StringColumn) and isinstance(b, str):
        return a.eq(b)                                   # one device pattern-match launch
    if isinstance(a, StringColumn) and isinstance(b, StringColumn) and len(a) == len(b):
        return a.eq_rows(None, b, None)                  # row-wise byte-exact equality (one device launch)
    ta, tb = _to_tensor_col(a), _to_tensor_col(b)
    if ta is not None and (tb is not None or not isinstance(b, (list, StringColumn, SelfRef))):
        other = tb if tb is not None else b
        if isinstance(other, torch.Tensor):
            other = other.to(ta.device)
        r = ta == other
        return r if r.dim() <= 1 else r.flatten(1).all(1)
    return _elementwise(lambda x, y: x == y, a, b)


def _logic(op, a, b):
    ta, tb = _to_tensor_col(a), _to_tensor_col(b)
    if ta is not None and tb is not None:
        tb = tb.to(ta.device)
        return (ta.bool() & tb.bool()) if op == "&&" else (ta.bool() | tb.bool())
    f = (lambda x, y: bool(x) and bool(y)) if op == "&&" else (lambda x, y: bool(x) or bool(y))
    return _elementwise(f, a, b)


def _not(a):
    t = _to_tensor_col(a)
    if t is not None:
        return ~t.bool()
    if isinstance(a, StringColumn):
        a = a.tolist()
    return [not x for x in a]


def _elementwise(f, a, b):
    if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
        return f(a, b.to(a.device))
    if isinstance(a, torch.Tensor) and not isinstance(b, (list, StringColumn, SelfRef)):
        return f(a, b)
    if isinstance(b, torch.Tensor) and not isinstance(a, (list, StringColumn, SelfRef)):
        return f(a, b)
    if isinstance(a, (list, StringColumn, torch.Tensor)) or isinstance(b, (list, StringColumn, torch.Tensor)):
        n = len(a) if isinstance(a, (list, StringColumn, torch.Tensor)) else len(b)
        ga, gb = _row_accessor(a), _row_accessor(b)
        return [f(ga(i), gb(i)) for i in range(n)]
    return f(a, b)


class Values(Lambda):
    """The [n, F] float64 value row of an aggregation from F scalar lambdas (column-major: each column is
    contiguous, as the device group-by reads it). Tree-built value rows compile into the fused pipeline kernel
    (execution/pipeline.py); the eager path stacks the columns."""

    kind = "values"

    def __init__(self, *items):
        super().__init__(children=[_lift(x) for x in items])

    def eval_node(self, inputs, child_vals):
        n, dev = _len_dev(child_vals)
        cols = []
        for v in child_vals:
            t = v if isinstance(v, torch.Tensor) else torch.as_tensor(v)
            t = t.to(dev, torch.float64)
            cols.append(t.expand(n) if t.dim() == 0 else t)
        return torch.stack(cols, 0).t()


class KeyTuple(Lambda):
    """A composite group / join key: a tuple of key columns (exact multi-column equality)."""

    kind = "keys"

    def __init__(self, *items):
        super().__init__(children=[_lift(x) for x in items])

    def eval_node(self, inputs, child_vals):
        return tuple(child_vals)


class Like(Lambda):
    """SQL ``LIKE`` of a string lambda against a pattern ('%' = any run, '_' = any byte)."""

    kind = "like"

    def __init__(self, x, pattern: str, negate: bool = False):
        super().__init__(children=[_lift(x)])
        self.pattern, self.negate = pattern, negate

    def eval_node(self, inputs, child_vals):
        v = child_vals[0]
        col = v if isinstance(v, StringColumn) else StringColumn.from_list(list(v))
        return col.like(self.pattern, self.negate)


class IsIn(Lambda):
    """``x IN (v1, v2, ...)`` over a string or numeric lambda."""

    kind = "isin"

    def __init__(self, x, values):
        super().__init__(children=[_lift(x)])
        self.values = list(values)

    def eval_node(self, inputs, child_vals):
        v = child_vals[0]
        if isinstance(v, StringColumn):
            return v.isin(self.values)
        if isinstance(v, torch.Tensor):
            return torch.isin(v, torch.tensor(self.values, dtype=v.dtype, device=v.device))
        s = set(self.values)
        return torch.tensor([x in s for x in v], dtype=torch.bool)


class Select(Lambda):
    """``cond ? a : b`` (SQL CASE WHEN cond THEN a ELSE b END)."""

    kind = "select"

    def __init__(self, cond, a, b):
        super().__init__(children=[_lift(cond), _lift(a), _lift(b)])

    def eval_node(self, inputs, child_vals):
        c, a, b = child_vals
        c = c if isinstance(c, torch.Tensor) else torch.as_tensor(c)
        a = a if isinstance(a, torch.Tensor) else torch.as_tensor(a, dtype=torch.float64)
        b = b if isinstance(b, torch.Tensor) else torch.as_tensor(b, dtype=torch.float64)
        return torch.where(c.bool(), a.to(c.device), b.to(c.device))


def _len_dev(vals):
    for v in vals:
        if isinstance(v, torch.Tensor) and v.dim() >= 1:
            return v.shape[0], v.device
        if isinstance(v, (list, StringColumn)):
            return len(v), getattr(v, "device", torch.device("cpu"))
    return 1, torch.device("cpu")


# --------------------------------------------------------------------- creation functions
def make_lambda_from_member(arg: Arg, member: str) -> Lambda:
    return AttAccess(arg, member)


def make_lambda_from_method(arg: Arg, method: str) -> Lambda:
    return MethodCall(arg, method)


def make_lambda_from_self(arg: Arg) -> Lambda:
    return SelfLambda(arg)


def make_lambda(*args, vectorized: bool = False, tag: Optional[str] = None) -> Lambda:
    """make_lambda(in1, [in2, ...], fn): the last positional argument is the function."""
    *ins, fn = args
    if not callable(fn):
        raise TypeError("make_lambda(..., fn): last argument must be callable")
    return Native(ins, fn, vectorized=vectorized, tag=tag)


def make_batch_lambda(*args, tag: Optional[str] = None) -> Lambda:
    """Vectorised native lambda: fn gets RecordBatch / column arguments."""
    return make_lambda(*args, vectorized=True, tag=tag)


# reference-style camelCase aliases
makeLambda = make_lambda
makeLambdaFromMember = make_lambda_from_member
makeLambdaFromMethod = make_lambda_from_method
makeLambdaFromSelf = make_lambda_from_self

__all__ = ["Arg", "Lambda", "Literal", "SelfLambda", "SelfRef", "AttAccess", "MethodCall", "Native", "Binary",
           "Unary", "Values", "KeyTuple", "Like", "IsIn", "Select", "make_lambda", "make_batch_lambda", "make_lambda_from_member", "make_lambda_from_method",
           "make_lambda_from_self", "makeLambda", "makeLambdaFromMember", "makeLambdaFromMethod",
           "makeLambdaFromSelf"]
