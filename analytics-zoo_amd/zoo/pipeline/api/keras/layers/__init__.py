"""zoo.pipeline.api.keras.layers — every Keras-1 layer of the reference (K3/K4)."""
from zoo.pipeline.api.keras.base import Input, InputLayer, Lambda, Layer, ZooKerasLayer
from zoo.pipeline.api.keras.engine.topology import Merge, merge
from zoo.pipeline.api.keras.layers.core import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.convolutional import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.pooling import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.normalization import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.recurrent import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.embeddings import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.advanced_activations import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.wrappers import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.torch_layers import *  # noqa: F401,F403
from zoo.pipeline.api.keras.layers.self_attention import TransformerLayer, BERT  # noqa: F401

# explicit export list: the reference-compatible submodule ``layers.torch`` must never
# leak into ``from zoo.pipeline.api.keras.layers import *`` and shadow the torch package
__all__ = [_n for _n in dir() if not _n.startswith("_") and _n != "torch"]
