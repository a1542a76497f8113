"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras2.layers.core`` (Py/pipeline/api/keras2/layers/core.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras2.layers import Dense, Activation, Dropout, Flatten  # noqa: F401
