"""Series (reference: python/pycylon/series.py:25-76): a named 1-D column."""
from typing import Any, List

import pyarrow as pa
import torch

from .data.arrow_bridge import to_cylon_type


class Series(object):
    def __init__(self, series_id: str = None, data=None, data_type=None):
        self._id = series_id or "0"
        if isinstance(data, torch.Tensor):
            self._data = data
            self._dtype = None
        else:
            arr = data if isinstance(data, (pa.Array, pa.ChunkedArray)) else pa.array(list(data) if data is not None
                                                                                     else [])
            if isinstance(arr, pa.ChunkedArray):
                arr = arr.combine_chunks()
            self._data = arr
            self._dtype = data_type if data_type is not None else to_cylon_type(arr.type)

    @property
    def id(self):
        return self._id

    @property
    def data(self):
        return self._data

    @property
    def dtype(self):
        if self._dtype is None and isinstance(self._data, torch.Tensor):
            return self._data.dtype
        return self._dtype

    @property
    def shape(self):
        return (len(self._data),)

    def __len__(self):
        return len(self._data)

    def __getitem__(self, item):
        if isinstance(self._data, torch.Tensor):
            return self._data[item]
        return self._data[item].as_py() if isinstance(item, int) else self._data[item]

    def to_list(self) -> List[Any]:
        if isinstance(self._data, torch.Tensor):
            return self._data.cpu().tolist()
        return self._data.to_pylist()

    def __repr__(self):
        return f"Series({self._id}, {self.to_list()[:10]})"
