from .datasets import (ArrayImageDataset, HashTokenizer, ImageFolderDataset, TextClassificationDataset,  # noqa: F401
                       synthetic_image_dataset)
from .image_classification import ImageClassificationModel  # noqa: F401
from .model_factory import get_model, get_supported_models, load_model  # noqa: F401
from .text_classification import TextClassificationModel  # noqa: F401
from .dataset_factory import get_dataset, load_dataset  # noqa: F401,E402
from .hugging_face import HuggingFaceTextClassificationDataset, HuggingFaceTextClassificationModel  # noqa: F401,E402
