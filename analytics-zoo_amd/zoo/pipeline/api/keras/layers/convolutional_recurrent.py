"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras.layers.convolutional_recurrent`` (Py/pipeline/api/keras/layers/convolutional_recurrent.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras.layers.recurrent import ConvLSTM2D, ConvLSTM3D  # noqa: F401
