from .api import DataAPI, DataAPIType, get_data_api  # noqa: F401
