"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras2.layers.convolutional`` (Py/pipeline/api/keras2/layers/convolutional.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras2.layers import Conv1D, Conv2D, Cropping1D  # noqa: F401
