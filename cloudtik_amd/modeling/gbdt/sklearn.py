"""scikit-learn style estimators over the GBDT booster (the XGBClassifier / XGBRegressor
surface the reference's xgboost modeling code uses)."""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np

from .booster import Booster, DMatrix


class _Base:
    _objective = "reg:squarederror"

    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.3, max_depth: int = 6,
                 early_stopping_rounds: Optional[int] = None, device=None, **params: Any):
        self.n_estimators = n_estimators
        self.early_stopping_rounds = early_stopping_rounds
        self.device = device
        self.params: Dict[str, Any] = dict(params, eta=learning_rate, max_depth=max_depth)
        self.params.setdefault("objective", self._objective)
        self.booster_: Optional[Booster] = None
        self.evals_result_: Dict = {}

    def _fit(self, X, y, sample_weight=None, eval_set=None, verbose=False):
        dtrain = DMatrix(X, y, sample_weight)
        evals = [(DMatrix(ex, ey), f"validation_{i}") for i, (ex, ey) in enumerate(eval_set or [])]
        self.booster_ = Booster(self.params, device=self.device).train(
            dtrain, self.n_estimators, evals, self.early_stopping_rounds, verbose, evals_result=self.evals_result_)
        return self

    def get_booster(self) -> Booster:
        return self.booster_

    @property
    def feature_importances_(self) -> np.ndarray:
        s = self.booster_.get_score("total_gain")
        v = np.array([s.get(n, 0.0) for n in self.booster_.feature_names], dtype=np.float32)
        return v / max(v.sum(), 1e-12)

    def save_model(self, path: str):
        self.booster_.save_model(path)


class GBDTRegressor(_Base):
    def fit(self, X, y, sample_weight=None, eval_set=None, verbose=False):
        return self._fit(X, y, sample_weight, eval_set, verbose)

    def predict(self, X) -> np.ndarray:
        return self.booster_.predict(X)


class GBDTClassifier(_Base):
    _objective = "binary:logistic"

    def fit(self, X, y, sample_weight=None, eval_set=None, verbose=False):
        y = np.asarray(y)
        self.classes_ = np.unique(y)
        if len(self.classes_) > 2:
            self.params["objective"] = "multi:softprob"
            self.params["num_class"] = len(self.classes_)
        y_idx = np.searchsorted(self.classes_, y).astype(np.float32)
        es = [(ex, np.searchsorted(self.classes_, np.asarray(ey)).astype(np.float32)) for ex, ey in (eval_set or [])]
        return self._fit(X, y_idx, sample_weight, es, verbose)

    def predict_proba(self, X) -> np.ndarray:
        p = self.booster_.predict(X)
        return np.stack([1 - p, p], axis=1) if p.ndim == 1 else p

    def predict(self, X) -> np.ndarray:
        return self.classes_[self.predict_proba(X).argmax(1)]
