"""Import-path compatibility with the reference module ``zoo.pipeline.api.keras.layers.torch`` (Py/pipeline/api/keras/layers/torch.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.keras.layers.advanced_activations import AddConstant, MulConstant, CAdd, CMul, Exp, Identity, Log, Mul, Power, Scale, Sqrt, Square, HardShrink, HardTanh, Negative, PReLU, RReLU, SoftShrink, BinaryThreshold, Threshold, GaussianSampler  # noqa: F401
from zoo.pipeline.api.keras.layers.convolutional import ShareConvolution2D, ResizeBilinear  # noqa: F401
from zoo.pipeline.api.keras.layers.normalization import LRN2D, WithinChannelLRN2D  # noqa: F401
from zoo.pipeline.api.keras.layers.torch_layers import Select, Narrow, Squeeze, SelectTable  # noqa: F401
