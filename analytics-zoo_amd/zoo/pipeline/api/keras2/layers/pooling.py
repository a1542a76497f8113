"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras2.layers.pooling`` (Py/pipeline/api/keras2/layers/pooling.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras2.layers import MaxPooling1D, AveragePooling1D, GlobalAveragePooling1D, GlobalMaxPooling1D, GlobalAveragePooling2D  # noqa: F401
