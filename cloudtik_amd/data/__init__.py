"""Data path of the AI runtime: Parquet / columnar host data -> native pinned-slot loader ->
hipMemcpyAsync on a side stream -> device batches."""
from .loader import NativeLoader  # noqa: F401
from .parquet import ParquetDataLoader, read_parquet_columns, write_parquet  # noqa: F401
