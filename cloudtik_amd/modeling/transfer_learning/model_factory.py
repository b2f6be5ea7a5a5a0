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


def get_model(model_name: str, framework: str = "pytorch", use_case: str = None, model_hub: str = None, **kwargs):
    """``model_hub="hugging_face"`` (or a local HF checkpoint directory) selects the HF text
    classifier (reference text_classification/pytorch/hugging_face)."""
    if framework != "pytorch":
        raise ValueError("only the pytorch framework is provided on this platform")
    import os
    from .hugging_face import HF_MODELS, HuggingFaceTextClassificationModel
    if use_case in (None, "text_classification") and (model_hub == "hugging_face" or os.path.isdir(model_name)
                                                      or (model_hub is None and model_name in HF_MODELS
                                                          and model_name not in ENCODERS)):
        return HuggingFaceTextClassificationModel(model_name, **kwargs)
    for uc, (cls, names) in USE_CASES.items():
        if (use_case in (None, uc)) and model_name in names:
            return cls(model_name, **kwargs)
    raise ValueError(f"no {use_case or 'any'} model named {model_name!r}; supported: {get_supported_models()}")


def load_model(output_dir: str, device=None):
    import json
    import os
    with open(os.path.join(output_dir, "model_config.json")) as f:
        meta = json.load(f)
    if meta.get("hub") == "hugging_face":
        from .hugging_face import HuggingFaceTextClassificationModel
        return HuggingFaceTextClassificationModel.load(output_dir, device=device)
    return USE_CASES[meta["use_case"]][0].load(output_dir, device=device)
