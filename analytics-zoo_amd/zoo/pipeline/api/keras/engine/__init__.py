from zoo.pipeline.api.keras.engine.topology import KerasNet, Model, Sequential, Merge, merge  # noqa: F401
from zoo.pipeline.api.keras.base import ZooKerasLayer, Input, InputLayer  # noqa: F401
