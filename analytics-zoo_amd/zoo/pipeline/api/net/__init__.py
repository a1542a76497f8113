from zoo.pipeline.api.net.graph_net import GraphNet, NodeLayer  # noqa: F401
from zoo.pipeline.api.net.net import Net  # noqa: F401
from zoo.pipeline.api.net.torch_net import TorchCriterion, TorchLayer, TorchModel, TorchNet  # noqa: F401
