from .catalog import Catalog
from .manager import DEFAULT_PAGE_SIZE, StorageManager
from .serde import deserialize_batch, serialize_batch
from .sets import DenseMatrixSet, Page, UserSet

__all__ = ["Catalog", "StorageManager", "DEFAULT_PAGE_SIZE", "serialize_batch", "deserialize_batch", "UserSet",
           "DenseMatrixSet", "Page"]
