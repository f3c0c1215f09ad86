from .record import (PDBObject, RecordBatch, RecordView, Tensor, Vector, batch_of, column_concat, column_item,
                     column_kind, column_take, lookup_type, make_column, register_type, registered_types)
from .builtin import *  # noqa: F401,F403
from .builtin import getter, vectorized

__all__ = ["PDBObject", "RecordBatch", "RecordView", "Tensor", "Vector", "batch_of", "lookup_type", "register_type",
           "registered_types", "getter", "vectorized", "make_column", "column_item", "column_take", "column_concat",
           "column_kind"]
