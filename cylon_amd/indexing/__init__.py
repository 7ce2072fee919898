"""cylon_amd.indexing (reference: python/pycylon/indexing/index.pyx, cpp/src/cylon/indexing/)."""
from .index import (BaseIndex, BinaryTreeIndex, BTreeIndex, HashIndex, ILocIndexer, IndexingSchema, LinearIndex, LocIndexer, PyLocIndexer,
                    RangeIndex, build_index)

__all__ = ["IndexingSchema", "BaseIndex", "LinearIndex", "HashIndex", "BinaryTreeIndex", "BTreeIndex", "RangeIndex", "build_index", "LocIndexer",
           "ILocIndexer", "PyLocIndexer"]
