"""Computation (UDF) classes — the netsDB/PlinyCompute programming model.

Reference: src/lambdas/headers/Computation.h, SelectionComp.h, MultiSelectionComp.h, JoinComp.h,
AggregateComp.h, ScanSet.h, SetWriter.h, PartitionComp.h; src/queryExecution/headers/
ClusterAggregateComp.h, TopKComp.h; src/builtInPDBObjects/headers/ScanUserSet.h, WriteUserSet.h.

Users subclass these and override the lambda factories (``get_selection``, ``get_projection``,
``get_key_projection``, ``get_value_projection``).  A graph of computations is compiled to TCAP
(:mod:`netsdb_amd.logical_plan.tcap`) and executed by the pipeline engine.

MI355X-native extension: a computation may declare a *tensor pattern* (``tensor_pattern()``)
describing the math its opaque lambda performs on MatrixBlock payloads (block matmul, bias+act,
row softmax, ...).  The physical planner uses it to lower join+aggregate chains over dense
matrix sets into fused MFMA kernels; without it the generic (still batched/vectorised) join,
aggregate and projection operators run.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import List, Optional

from ..lambdas import Arg, Lambda, Literal

_ids = itertools.count()


class Computation:
    num_inputs = 1
    comp_type = "Computation"

    def __init__(self):
        self.inputs: List[Optional[Computation]] = [None] * self.num_inputs
        self.uid = next(_ids)
        self.batch_size = 0
        self.output_type: Optional[type] = None
        self.input_types: List[Optional[type]] = [None] * self.num_inputs

    # --- graph wiring (reference: setInput(i, comp) / setInput(comp))
    def set_input(self, *args):
        if len(args) == 1:
            i, comp = 0, args[0]
        else:
            i, comp = args
        if i >= self.num_inputs:
            raise IndexError(f"{self.comp_type} has {self.num_inputs} inputs")
        self.inputs[i] = comp
        return self

    setInput = set_input

    def get_input(self, i=0):
        return self.inputs[i]

    def get_computation_type(self) -> str:
        return self.comp_type

    def get_num_inputs(self) -> int:
        return self.num_inputs

    def extract_lambdas(self) -> dict:
        """name -> Lambda node for every lambda of this computation (named during TCAP compile)."""
        return getattr(self, "_lambdas", {})

    def tensor_pattern(self):
        return None

    def needs_materialize_output(self) -> bool:
        return False

    def set_batch_size(self, n: int):
        self.batch_size = n

    def args(self) -> List[Arg]:
        return [Arg(i, t) for i, t in enumerate(self.input_types)]

    def __repr__(self):
        return f"{self.comp_type}_{self.uid}"


# ----------------------------------------------------------------------------- sources/sinks
class ScanSet(Computation):
    """ScanUserSet<T>(db, set)."""

    num_inputs = 0
    comp_type = "ScanUserSet"

    def __init__(self, db: str, set_name: str, type_: Optional[type] = None):
        super().__init__()
        self.db, self.set_name = db, set_name
        self.output_type = type_


ScanUserSet = ScanSet


class WriteSet(Computation):
    """WriteUserSet<T>(db, set) — the pipeline sink that materialises into a stored set."""

    comp_type = "WriteUserSet"

    def __init__(self, db: str, set_name: str, type_: Optional[type] = None):
        super().__init__()
        self.db, self.set_name = db, set_name
        self.output_type = type_

    def needs_materialize_output(self):
        return True


WriteUserSet = WriteSet


# ----------------------------------------------------------------------------- selection
class SelectionComp(Computation):
    """filter (get_selection) + per-record map (get_projection)."""

    comp_type = "SelectionComp"

    def get_selection(self, in0: Arg) -> Lambda:
        return Literal(True)

    def get_projection(self, in0: Arg) -> Lambda:
        raise NotImplementedError

    getSelection = get_selection
    getProjection = get_projection


class MultiSelectionComp(SelectionComp):
    """filter + one-to-many map: get_projection returns a list per record (FLATTEN)."""

    comp_type = "MultiSelectionComp"


class JoinComp(Computation):
    """N-way join: get_selection(*ins) must be a conjunction of equalities for a hash join
    (otherwise a cartesian product is filtered); get_projection(*ins) builds the output."""

    comp_type = "JoinComp"

    def __init__(self, num_inputs: int = 2):
        self.num_inputs = num_inputs
        super().__init__()

    def get_selection(self, *ins: Arg) -> Lambda:
        raise NotImplementedError

    def get_projection(self, *ins: Arg) -> Lambda:
        raise NotImplementedError

    getSelection = get_selection
    getProjection = get_projection


class AggregateComp(Computation):
    """Group-by: key = get_key_projection(in), value = get_value_projection(in); values with
    the same key are combined with ``combine`` (default ``+``, tensor-aware)."""

    comp_type = "AggregationComp"

    def get_key_projection(self, in0: Arg) -> Lambda:
        raise NotImplementedError

    def get_value_projection(self, in0: Arg) -> Lambda:
        raise NotImplementedError

    getKeyProjection = get_key_projection
    getValueProjection = get_value_projection

    def combine(self, a, b):
        return a + b

    # vectorised combine: 'sum' | 'max' | 'min' | None (use combine())
    reduce_op: Optional[str] = "sum"

    def make_output(self, keys, values):
        """Build the output batch from per-group key and value columns (default: tuple set)."""
        from ..objects.record import RecordBatch

        if isinstance(keys, tuple):
            cols = {f"key{i}": k for i, k in enumerate(keys)}
        else:
            cols = {"key": keys}
        cols["value"] = values
        return RecordBatch(cols, len(values))

    def needs_materialize_output(self):
        return True


ClusterAggregateComp = AggregateComp


class PartitionComp(Computation):
    """Re-partition the input across nodes by a key lambda and store it (reference PartitionComp)."""

    comp_type = "PartitionComp"

    def __init__(self, db: str = "", set_name: str = ""):
        super().__init__()
        self.db, self.set_name = db, set_name

    def get_key_projection(self, in0: Arg) -> Lambda:
        raise NotImplementedError

    def get_projection(self, in0: Arg) -> Lambda:
        from ..lambdas import SelfLambda

        return SelfLambda(in0)

    def needs_materialize_output(self):
        return True


class TopKComp(Computation):
    """Top-k by score (reference queryExecution/headers/TopKComp.h)."""

    comp_type = "TopKComp"

    def __init__(self, k: int = 10):
        super().__init__()
        self.k = k

    def get_value_projection(self, in0: Arg) -> Lambda:
        raise NotImplementedError

    def get_key_projection(self, in0: Arg) -> Lambda:
        from ..lambdas import SelfLambda

        return SelfLambda(in0)


# ----------------------------------------------------------------------------- tensor patterns
@dataclass
class BlockMatmul:
    """join(A.blockCol == B.blockCol [or B.blockRow]) projecting A.data @ B.data(^T) — the
    netsDB block-matmul join (FFTransposeMult, LASillyMultiply1Join, LASillyTransposeMultiply1Join)."""

    transpose_a: bool = False
    transpose_b: bool = True
    a_input: int = 0
    b_input: int = 1


@dataclass
class BlockSum:
    """aggregate whose key is the block (row, col) and value the payload summed (FFAggMatrix)."""


@dataclass
class BiasAct:
    """join(X.blockRow == bias.blockRow) projecting act(X + bias) (FFReluBiasSum & friends)."""

    act: str = "relu"
    dropout: float = 0.0
    bias_along: str = "row"     # bias indexed by the data's row ("row") or column ("col")
    transpose_out: bool = False
    data_input: int = 0
    bias_input: int = 1
    seed: int = 0


@dataclass
class RowSoftmax:
    """RowAggregate(sum exp) + OutputLayer(divide): softmax over each row of a matrix set."""


@dataclass
class Elementwise:
    """join(A.key == B.key) projecting op(A.data, B.data) blockwise (LASillyAddJoin, ...Substract,
    ...ScaleMultiply)."""

    op: str = "add"
    extra: dict = field(default_factory=dict)


@dataclass
class GateSum:
    """N-way join(equal block keys) projecting act(in_0 + ... + in_{n-1}) (LSTMThreeWaySum)."""

    act: str = "sigmoid"


@dataclass
class CellUpdate:
    """4-way join projecting f * c_prev + i * g (LSTMTwoSum; inputs f, c_prev, i, g)."""


@dataclass
class HiddenOut:
    """2-way join projecting o * tanh(c) (LSTMHiddenState; inputs o, c)."""


@dataclass
class Transpose:
    """selection swapping block indices and transposing payloads (LASillyTransposeSelection)."""


@dataclass
class Scale:
    """selection multiplying every block by a constant (the LA DSL's ``c * A``; LAParser.y numeric literals with
    the block-wise pattern of LASillyScaleMultiplyJoin)."""

    scalar: float = 1.0


@dataclass
class Reduce:
    """aggregate reducing a matrix along rows ('row' -> column vector), columns ('col' -> row vector)
    or everything ('all' -> 1x1) with max/min/sum (LASillyRow/Col/Max/MinElement/...Aggregate)."""

    axis: str = "row"
    op: str = "sum"


@dataclass
class Inverse:
    """matrix inverse (LASillyInverse1Aggregate + Inverse2Selection + Inverse3MultiSelection)."""


@dataclass
class Duplicate:
    """multi-selection repeating a row vector down ('row') or a column vector across ('col')
    (LASillyDuplicateRowMultiSelection / DuplicateColMultiSelection)."""

    axis: str = "row"
    block_size: int = 1
    num_blocks: int = 1


__all__ = ["Computation", "ScanSet", "ScanUserSet", "WriteSet", "WriteUserSet", "SelectionComp",
           "MultiSelectionComp", "JoinComp", "AggregateComp", "ClusterAggregateComp", "PartitionComp", "TopKComp",
           "BlockMatmul", "BlockSum", "BiasAct", "RowSoftmax", "Elementwise", "Transpose", "Scale", "Reduce", "Inverse",
           "Duplicate"]
