"""Model factory (reference modeling/transfer_learning/model_factory.py:137): pick a model
by (framework, use case, name)."""
from __future__ import annotations

from typing import Dict, List

from .anomaly_detection import ImageAnomalyDetectionModel
from .image_classification import BACKBONES, ImageClassificationModel
from .text_classification import ENCODERS, TextClassificationModel

USE_CASES = {"image_classification": (ImageClassificationModel, BACKBONES),
             "text_classification": (TextClassificationModel, ENCODERS),
             "image_anomaly_detection": (ImageAnomalyDetectionModel, BACKBONES)}


def get_supported_models(framework: str = "pytorch", use_case: str = None) -> Dict[str, List[str]]:
    if framework != "pytorch":
        return {}
    return {uc: sorted(names) for uc, (_, names) in USE_CASES.items() if use_case in (None, uc)}


def get_model(model_name: str, framework: str = "pytorch", use_case: str = None, **kwargs):
    if framework != "pytorch":
        raise ValueError("only the pytorch framework is provided on this platform")
    for uc, (cls, names) in USE_CASES.items():
        if (use_case in (None, uc)) and model_name in names:
            return cls(model_name, **kwargs)
    raise ValueError(f"no {use_case or 'any'} model named {model_name!r}; supported: {get_supported_models()}")


def load_model(output_dir: str, device=None):
    import json
    import os
    with open(os.path.join(output_dir, "model_config.json")) as f:
        uc = json.load(f)["use_case"]
    return USE_CASES[uc][0].load(output_dir, device=device)
