"""Data loading and mini-batching for ML pipelines (reference:
python/pycylon/util/data/DataManager.py:33-169, cpp/src/tutorial/demo_pytorch*.py).

MI355X-native difference: batches are handed to torch as device tensors that
alias the table's HBM buffers (no to_numpy / host hop as in the reference demo)."""
import math
import os
from typing import List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv
import torch


class Partition(object):
    def __init__(self, data, index):
        self.data = data
        self.index = index

    def __len__(self):
        return len(self.index)

    def __getitem__(self, index):
        return self.data[self.index[index]]


class DataLoader(object):
    def __init__(self, source_dir: str = None, source_files: Optional[List] = None,
                 source_file_names: Optional[List[str]] = None, file_type: str = "csv", loader_type: str = "arrow",
                 delimiter: str = ","):
        self._source_dir = source_dir
        self._source_files = list(source_files or [])
        self._source_file_names = list(source_file_names or [])
        self._file_type = file_type
        self.loader_type = loader_type
        self._delimiter = delimiter
        self._dataset: List = []

    @property
    def source_dir(self) -> str:
        return self._source_dir

    @property
    def source_files(self) -> List[str]:
        return self._source_files

    @property
    def source_file_names(self) -> List[str]:
        return self._source_file_names

    @property
    def file_type(self) -> str:
        return self._file_type

    @property
    def delimiter(self) -> str:
        return self._delimiter

    @property
    def dataset(self) -> List:
        return self._dataset

    @dataset.setter
    def dataset(self, values: List):
        self._dataset = values

    def load(self):
        raise NotImplementedError(f"{type(self).__name__}.load: subclasses provide the loading strategy")


class LocalDataLoader(DataLoader):
    def load(self):
        if self.loader_type not in ("arrow", "cylon"):
            raise NotImplementedError(f"The Loader Type {self.loader_type} is not supported!")
        out = []
        for i, f in enumerate(self.source_files):
            path = os.path.join(self.source_dir or "", f)
            self._source_file_names.append(f"source_file_{i}")
            out.append(pacsv.read_csv(path, parse_options=pacsv.ParseOptions(delimiter=self.delimiter)))
        self.dataset = out
        return out


class DistributedDataLoader(DataLoader):
    """Each rank loads the files assigned to it round-robin (file i -> rank i % world)."""

    def __init__(self, ctx, **kw):
        super().__init__(**kw)
        self._ctx = ctx

    def load(self):
        from ..io import read_csv
        r, w = self._ctx.get_rank(), self._ctx.get_world_size()
        mine = [f for i, f in enumerate(self.source_files) if i % w == r]
        self.dataset = [read_csv(self._ctx, os.path.join(self.source_dir or "", f)) for f in mine]
        return self.dataset


class MiniBatcher(object):
    @staticmethod
    def generate_minibatches(data=None, minibatch_size: int = 1):
        """Split rows into ceil(n / b) batches of exactly b rows; the last batch is padded by
        re-using randomly chosen earlier rows (the reference's documented intent)."""
        if isinstance(data, torch.Tensor):
            n = data.shape[0]
            nb = math.ceil(n / float(minibatch_size))
            pad = nb * minibatch_size - n
            if pad:
                extra = torch.randint(0, n, (pad,), device=data.device)
                data = torch.cat([data, data[extra]])
            return data.reshape(nb, minibatch_size, *data.shape[1:])
        arr = np.asarray(data)
        n = arr.shape[0]
        nb = math.ceil(n / float(minibatch_size))
        pad = nb * minibatch_size - n
        if pad:
            arr = np.concatenate([arr, arr[np.random.randint(0, n, pad)]])
        return arr.reshape(nb, minibatch_size, *arr.shape[1:])

    @staticmethod
    def table_batches(table, columns: List[str], batch_size: int):
        """Yield [batch, len(columns)] float tensors on the table's device (zero-copy column views)."""
        cols = table.to_torch()
        mat = torch.stack([cols[c].to(torch.float32) for c in columns], dim=1)
        for s in range(0, mat.shape[0], batch_size):
            yield mat[s:s + batch_size]
