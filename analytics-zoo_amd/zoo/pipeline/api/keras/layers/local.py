"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras.layers.local`` (Py/pipeline/api/keras/layers/local.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras.layers.convolutional import LocallyConnected1D, LocallyConnected2D  # noqa: F401
