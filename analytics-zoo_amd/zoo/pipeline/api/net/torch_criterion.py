"""Import-path compatibility with the reference module ``zoo.pipeline.api.net.torch_criterion`` (Py/pipeline/api/net/torch_criterion.py):
the implementations live in the modules imported below."""
from zoo.pipeline.api.net.torch_net import TorchCriterion  # noqa: F401
