"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras.layers.noise`` (Py/pipeline/api/keras/layers/noise.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras.layers.advanced_activations import GaussianNoise, GaussianDropout  # noqa: F401
