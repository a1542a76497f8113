"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras2.layers.local`` (Py/pipeline/api/keras2/layers/local.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras2.layers import LocallyConnected1D  # noqa: F401
