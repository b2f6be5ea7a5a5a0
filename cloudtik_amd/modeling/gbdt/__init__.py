from .booster import BinMapper, Booster, BoostParams, DMatrix, evaluate_metric, train  # noqa: F401
from .sklearn import GBDTClassifier, GBDTRegressor  # noqa: F401
