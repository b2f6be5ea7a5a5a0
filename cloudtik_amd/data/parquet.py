"""Parquet -> columnar host arrays -> NativeLoader (the AI half of the Spark + AI pipeline:
Spark writes Parquet to HDFS / local FS, training ranks stream it to the GPU; reference:
Horovod-on-Spark ``Store`` -> Parquet -> Petastorm readers, examples/runtime/ai/basics/
pytorch/mnist-pytorch-spark-horovod-hyperopt-mlflow.py:159,200-214).

Scalar numeric columns become 1-D arrays; fixed-size list columns (e.g. flattened images
or token ids) become [rows, n] arrays, optionally reshaped with ``shapes={"image": (3, 224, 224)}``.
``hdfs://`` and other fsspec URLs are read through pyarrow's filesystem layer when available.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np


def _expand(paths: Union[str, Sequence[str]]) -> List[str]:
    if isinstance(paths, str):
        paths = [paths]
    out = []
    for p in paths:
        if "://" in p:
            out.append(p)
        elif os.path.isdir(p):
            out += sorted(glob.glob(os.path.join(p, "**", "*.parquet"), recursive=True))
        else:
            out += sorted(glob.glob(p)) or [p]
    return out


def _column_to_numpy(col) -> np.ndarray:
    import pyarrow as pa
    col = col.combine_chunks() if isinstance(col, pa.ChunkedArray) else col
    t = col.type
    if pa.types.is_fixed_size_binary(t):
        # raw row bytes (images): one memcpy-free view of the values buffer
        w = t.byte_width
        buf = col.buffers()[1]
        return np.frombuffer(buf, dtype=np.uint8, count=(col.offset + len(col)) * w).reshape(-1, w)[col.offset:]
    if pa.types.is_fixed_size_list(t) or pa.types.is_list(t) or pa.types.is_large_list(t):
        values = col.flatten().to_numpy(zero_copy_only=False)
        n = len(col)
        if n == 0:
            return values.reshape(0, 0)
        if pa.types.is_fixed_size_list(t):
            return values.reshape(n, t.list_size)
        offs = col.offsets.to_numpy()
        widths = np.diff(offs)
        if not (widths == widths[0]).all():
            raise ValueError("variable-length list columns are not supported by the batch loader")
        return values.reshape(n, int(widths[0]))
    return col.to_numpy(zero_copy_only=False)


def read_parquet_columns(paths, columns: Optional[Sequence[str]] = None,
                         shapes: Optional[Dict[str, Tuple[int, ...]]] = None,
                         dtypes: Optional[Dict[str, object]] = None) -> Dict[str, np.ndarray]:
    import pyarrow.parquet as pq
    tables = []
    for p in _expand(paths):
        if "://" in p:
            import pyarrow.fs as pafs
            fs, path = pafs.FileSystem.from_uri(p)
            tables.append(pq.read_table(path, columns=columns, filesystem=fs))
        else:
            tables.append(pq.read_table(p, columns=columns))
    if not tables:
        raise FileNotFoundError(f"no parquet files under {paths}")
    import pyarrow as pa
    table = pa.concat_tables(tables) if len(tables) > 1 else tables[0]
    out = {}
    for name in (columns or table.column_names):
        arr = _column_to_numpy(table.column(name))
        if dtypes and name in dtypes:
            arr = arr.astype(dtypes[name], copy=False)
        if shapes and name in shapes:
            arr = arr.reshape((arr.shape[0],) + tuple(shapes[name]))
        out[name] = np.ascontiguousarray(arr)
    return out


def write_parquet(path: str, columns: Dict[str, np.ndarray], row_group_size: int = 65536):
    """Write numpy columns ([rows] or [rows, ...] -> fixed-size list) to one Parquet file."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    arrays, names, dict_cols = [], [], []
    for name, a in columns.items():
        a = np.ascontiguousarray(a)
        if a.ndim == 1:
            arrays.append(pa.array(a))
            dict_cols.append(name)
        elif a.dtype == np.uint8:
            # uint8 tensors (images) as fixed-size binary rows: Parquet stores them as plain
            # byte arrays, so reading is a copy, not a per-element level decode (~50x faster
            # than a list<uint8> column for 224x224x3 images)
            flat = a.reshape(a.shape[0], -1)
            w = flat.shape[1]
            arrays.append(pa.FixedSizeBinaryArray.from_buffers(pa.binary(w), len(flat),
                                                               [None, pa.py_buffer(flat.reshape(-1))]))
        else:
            flat = a.reshape(a.shape[0], -1)
            arrays.append(pa.FixedSizeListArray.from_arrays(pa.array(flat.reshape(-1)), flat.shape[1]))
            dict_cols.append(name)
        names.append(name)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    pq.write_table(pa.Table.from_arrays(arrays, names=names), path, row_group_size=row_group_size,
                   use_dictionary=dict_cols)


class ParquetDataLoader:
    """read_parquet_columns + NativeLoader."""

    def __init__(self, paths, batch_size: int, columns: Optional[Sequence[str]] = None,
                 shapes: Optional[Dict[str, Tuple[int, ...]]] = None, dtypes: Optional[Dict[str, object]] = None,
                 **loader_kw):
        from cloudtik_amd.data.loader import NativeLoader
        self.columns = read_parquet_columns(paths, columns, shapes, dtypes)
        self.loader = NativeLoader(self.columns, batch_size, **loader_kw)

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        return iter(self.loader)

    def set_epoch(self, epoch: int):
        self.loader.set_epoch(epoch)
