"""Built-in PDB types (reference: src/builtInPDBObjects/headers, src/sharedLibraries/headers,
src/FF/headers/FFMatrixBlock.h / FFMatrixMeta.h / FFMatrixData.h, src/conv2d_memory_fusion/headers).

Methods that UDF lambdas call (``makeLambdaFromMethod(in, getBlockRowIndex)``) are declared with
:func:`getter` / :func:`vectorized`, so the engine evaluates them on a whole column at once
instead of object-at-a-time.
"""
from __future__ import annotations

import math
from typing import Callable

import torch

from .record import PDBObject, RecordBatch, Tensor, Vector


def vectorized(batch_fn: Callable[[RecordBatch], object]):
    """Decorate a per-record method with a whole-batch implementation ``batch_fn(batch)``."""

    def deco(fn):
        fn.__vectorized__ = batch_fn
        return fn

    return deco


def getter(field: str):
    """A method returning one field, evaluated as a column read."""

    def m(self):
        return getattr(self, field)

    m.__vectorized__ = lambda b: b.columns[field]
    m.__field__ = field
    return m


# ----------------------------------------------------------------- matrix blocks
class MatrixBlock(PDBObject):
    """A block of a block-partitioned matrix (LA DSL MatrixBlock / FF FFMatrixBlock).

    ``data`` is the [row_nums, col_nums] payload; in device-resident sets it is a view of an HBM
    page and blocks of one set are stacked into a single [nblocks, rows, cols] tensor.
    """

    block_row: int
    block_col: int
    row_nums: int
    col_nums: int
    total_rows: int
    total_cols: int
    data: Tensor()

    getBlockRowIndex = getter("block_row")
    getBlockColIndex = getter("block_col")
    getRowNums = getter("row_nums")
    getColNums = getter("col_nums")
    getTotalRowNums = getter("total_rows")
    getTotalColNums = getter("total_cols")

    def getKey(self):
        return (self.block_row, self.block_col)

    getKey.__vectorized__ = lambda b: (b.columns["block_row"], b.columns["block_col"])

    def getRowKey(self):
        return (self.block_row, 0)

    getRowKey.__vectorized__ = lambda b: (b.columns["block_row"], torch.zeros_like(b.columns["block_row"]))

    def getColKey(self):
        return (0, self.block_col)

    getColKey.__vectorized__ = lambda b: (torch.zeros_like(b.columns["block_col"]), b.columns["block_col"])

    def getValue(self):
        return self.data

    getValue.__vectorized__ = lambda b: b.columns["data"]

    def num_row_blocks(self):
        return math.ceil(self.total_rows / self.row_nums)

    def num_col_blocks(self):
        return math.ceil(self.total_cols / self.col_nums)

    def is_last_row_block(self):
        return self.block_row == self.num_row_blocks() - 1

    def is_last_col_block(self):
        return self.block_col == self.num_col_blocks() - 1


class FFMatrixBlock(MatrixBlock):
    """src/FF/headers/FFMatrixBlock.h (adds the distinct block id used by deduplication)."""

    distinct_block_id: int
    partition_by_col: bool


class MatrixMeta(PDBObject):
    block_row: int
    block_col: int
    total_rows: int
    total_cols: int


class TensorBlockMeta(PDBObject):
    """src/builtInPDBObjects/headers/TensorBlockMeta.h — n-d block index."""

    index: Vector(int)
    block_shape: Vector(int)


class TensorBlock(PDBObject):
    """n-dimensional tensor block (TensorBlockIdentifier + payload)."""

    block_id: int
    index: Vector(int)
    data: Tensor()


# ----------------------------------------------------------------- images (conv2d)
class Image(PDBObject):
    """conv2d_memory_fusion Image / Kernel: one [C,H,W] tensor with an id."""

    key: int
    channels: int
    height: int
    width: int
    data: Tensor()

    getKey = getter("key")


class Kernel(Image):
    pass


class ImageChunk(PDBObject):
    """conv2d_memory_fusion ImageChunk: a slab of im2col rows of one image."""

    image_key: int
    chunk_index: int
    data: Tensor()


# ----------------------------------------------------------------- relational test types
class Employee(PDBObject):
    name: str
    age: int
    department: str
    salary: float

    getName = getter("name")
    getAge = getter("age")
    getSalary = getter("salary")
    getDepartment = getter("department")


class Supervisor(PDBObject):
    me: object  # Employee
    team: list  # list of Employees

    def getMe(self):
        return self.me

    def getTeam(self):
        return self.team


class StringIntPair(PDBObject):
    myString: str
    myInt: int

    getString = getter("myString")
    getInt = getter("myInt")


class DoubleVector(PDBObject):
    data: Tensor()

    def getRawData(self):
        return self.data

    getRawData.__vectorized__ = lambda b: b.columns["data"]


class SumResult(PDBObject):
    identifier: int
    total: float

    getKey = getter("identifier")
    getValue = getter("total")


class DepartmentTotal(PDBObject):
    department: str
    total: float


class IntVal(PDBObject):
    value: int

    getValue = getter("value")


__all__ = [n for n in dir() if not n.startswith("_")]
