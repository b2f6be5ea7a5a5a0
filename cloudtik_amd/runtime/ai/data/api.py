"""Data API: one pandas-style namespace over pandas / pyspark.pandas / modin (reference
runtime/ai/data/api.py:27-69), so data-processing code switches engines by name.
"""
from __future__ import annotations

import enum
import importlib
from typing import Optional, Union

_MODULES = {"pandas": "pandas", "spark": "pyspark.pandas", "modin": "modin.pandas"}


class DataAPIType(enum.Enum):
    PANDAS = "pandas"
    SPARK = "spark"
    MODIN = "modin"

    def __str__(self):
        return self.value

    @staticmethod
    def from_str(name: str) -> "DataAPIType":
        try:
            return DataAPIType(name.lower())
        except ValueError:
            raise ValueError(f"unsupported data API {name!r} (choose from {[e.value for e in DataAPIType]})") \
                from None


class DataAPI:
    def __init__(self, api_type: Union[DataAPIType, str] = DataAPIType.PANDAS):
        self.api_type = DataAPIType.from_str(api_type) if isinstance(api_type, str) else api_type

    def pandas(self):
        """The pandas-compatible module of the engine (imported on first use)."""
        return importlib.import_module(_MODULES[self.api_type.value])

    def pandas_api(self):
        return self.pandas

    @property
    def native(self) -> bool:
        return self.api_type is DataAPIType.PANDAS

    def available(self) -> bool:
        try:
            self.pandas()
            return True
        except ImportError:
            return False


def get_data_api(api_type: Optional[Union[DataAPIType, str]] = None) -> DataAPI:
    return DataAPI(api_type or DataAPIType.PANDAS)
