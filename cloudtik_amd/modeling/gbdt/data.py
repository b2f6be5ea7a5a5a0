"""Config-driven tabular preprocessing for the GBDT workflow (reference
xgboost/modeling/data/{data_transform,data_splitting,post_transform,process}.py and
config/data-processing-config.yaml).

Transforms run in order on a pandas(-compatible) DataFrame, picked by the Data API
(``runtime.ai.data``).  Condition / variable expressions in the config (``'df.year > 2018'``,
``'df.loc[df["split"] == 0, "card_id"]'``) are Python expressions over ``df``, ``tmp``
(variables defined earlier), ``np`` and ``pd``; like a job script, the config is code the
user supplies and is evaluated with no builtins available.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

import numpy as np

log = logging.getLogger(__name__)


def _expr(expr: str, df, tmp: Dict[str, Any]):
    import pandas as pd
    return eval(compile(str(expr), "<data-config>", "eval"), {"__builtins__": {}},
                {"df": df, "tmp": tmp, "np": np, "pd": pd})


class DataTransformer:
    def __init__(self, df, tmp: Optional[Dict[str, Any]] = None):
        self.df = df
        self.tmp = tmp if tmp is not None else {}

    # ---------------------------------------------------------------- steps
    def normalize_feature_names(self, steps: List[Dict[str, Any]]):
        cols = list(self.df.columns)
        for step in steps:
            for k, v in step.items():
                if k == "replace_chars":
                    for a, b in v.items():
                        cols = [c.replace(a, b) for c in cols]
                elif k == "lowercase" and v:
                    cols = [c.lower() for c in cols]
        self.df.columns = cols

    def categorify(self, mapping: Dict[str, str]):
        for src, dst in mapping.items():
            self.df[dst] = self.df[src].astype("category").cat.codes

    def strip_chars(self, mapping: Dict[str, Dict[str, str]]):
        for dst, spec in mapping.items():
            for src, chars in spec.items():
                self.df[dst] = self.df[src].astype(str).str.replace(chars, "", regex=False)

    def combine_cols(self, mapping: Dict[str, Dict[str, List[str]]]):
        for dst, spec in mapping.items():
            cols = spec.get("concatenate_strings", [])
            out = self.df[cols[0]].astype(str)
            for c in cols[1:]:
                out = out + self.df[c].astype(str)
            self.df[dst] = out

    def time_to_seconds(self, mapping: Dict[str, str]):
        import pandas as pd
        for src, dst in mapping.items():
            t = pd.to_timedelta(self.df[src].astype(str).where(self.df[src].astype(str).str.count(":") == 2,
                                                               self.df[src].astype(str) + ":00"))
            self.df[dst] = t.dt.total_seconds()

    def change_datatype(self, mapping: Dict[str, Any]):
        for col, types in mapping.items():
            for t in (types if isinstance(types, list) else [types]):
                self.df[col] = self.df[col].astype(t)

    def min_max_normalization(self, mapping: Dict[str, str]):
        for src, dst in mapping.items():
            c = self.df[src].astype("float64")
            lo, hi = c.min(), c.max()
            self.df[dst] = (c - lo) / (hi - lo) if hi > lo else 0.0

    def one_hot_encoding(self, mapping: Dict[str, bool]):
        import pandas as pd
        for col, drop in mapping.items():
            d = pd.get_dummies(self.df[col], prefix=col, dtype=np.float32)
            self.df = pd.concat([self.df.drop(columns=[col]) if drop else self.df, d], axis=1)

    def string_to_list(self, mapping: Dict[str, Dict[str, str]]):
        for dst, spec in mapping.items():
            for src, sep in spec.items():
                self.df[dst] = self.df[src].fillna("").astype(str).str.split(sep)

    def multi_hot_encoding(self, mapping: Dict[str, bool]):
        import pandas as pd
        for col, drop in mapping.items():
            d = self.df[col].explode().str.get_dummies().groupby(level=0).max().add_prefix(f"{col}_")
            d = d.drop(columns=[c for c in d.columns if c == f"{col}_"], errors="ignore").astype(np.float32)
            self.df = pd.concat([self.df.drop(columns=[col]) if drop else self.df, d], axis=1)

    def add_constant_feature(self, mapping: Dict[str, Any]):
        for col, v in mapping.items():
            self.df[col] = v

    def modify_on_conditions(self, mapping: Dict[str, Dict[str, Any]]):
        for col, conds in mapping.items():
            for cond, value in conds.items():
                self.df.loc[_expr(cond, self.df, self.tmp), col] = value

    def define_variable(self, mapping: Dict[str, str]):
        for name, expr in mapping.items():
            self.tmp[name] = _expr(expr, self.df, self.tmp)

    def drop_columns(self, cols: List[str]):
        self.df = self.df.drop(columns=list(cols), errors="ignore")

    def apply(self, steps: List[Dict[str, Any]]):
        for step in steps or []:
            for name, arg in step.items():
                fn = getattr(self, name, None)
                if fn is None or name.startswith("_") or name == "apply":
                    raise ValueError(f"unknown data transform {name!r}")
                fn(arg)
        return self.df


def split_data(df, config: Dict[str, Any], tmp=None, seed: int = 0) -> Dict[str, Any]:
    """custom_rules: {name: condition} or random_split: {test_ratio}."""
    if not config:
        return {"train": df}
    if "custom_rules" in config:
        return {name: df[_expr(cond, df, tmp or {})] for name, cond in config["custom_rules"].items()}
    if "random_split" in config:
        r = float(config["random_split"].get("test_ratio", 0.1))
        mask = np.random.default_rng(seed).random(len(df)) < r
        return {"train": df[~mask], "test": df[mask]}
    raise ValueError(f"unknown data_splitting config {list(config)}")


def target_encoding(splits: Dict[str, Any], target_col: str, feature_cols: List[str], smoothing: float = 0.001):
    """Smoothed mean target per category, fitted on 'train', applied to every split."""
    tr = splits["train"]
    prior = float(tr[target_col].mean())
    for c in feature_cols:
        stats = tr.groupby(c, observed=True)[target_col].agg(["sum", "count"])
        enc = (stats["sum"] + prior * smoothing) / (stats["count"] + smoothing)
        for name, d in splits.items():
            d = d.copy()
            d[c] = d[c].map(enc).astype("float64").fillna(prior)
            splits[name] = d
    return splits


def process_data(df, config: Dict[str, Any], seed: int = 0) -> Dict[str, Any]:
    t = DataTransformer(df)
    df = t.apply(config.get("data_transform", []))
    splits = split_data(df, config.get("data_splitting", {}), t.tmp, seed)
    for step in config.get("post_transform", []) or []:
        for name, arg in step.items():
            if name == "target_encoding":
                splits = target_encoding(splits, arg["target_col"], arg["feature_cols"], arg.get("smoothing", 0.001))
            else:
                raise ValueError(f"unknown post transform {name!r}")
    return splits


def read_table(path: str, data_api: str = "pandas"):
    from cloudtik_amd.runtime.ai.data import get_data_api
    pd = get_data_api(data_api).pandas()
    if path.endswith(".parquet") or path.endswith("/"):
        return pd.read_parquet(path)
    return pd.read_csv(path)


def feature_frame(df, target_col: str, ignore_cols: Optional[List[str]] = None):
    drop = [target_col] + [c for c in (ignore_cols or []) if c in df.columns]
    X = df.drop(columns=drop)
    for c in X.columns:
        if str(X[c].dtype) in ("category", "object", "string"):
            X[c] = X[c].astype("category").cat.codes.astype("float32")
    return X.astype("float32"), df[target_col].astype("float32")
